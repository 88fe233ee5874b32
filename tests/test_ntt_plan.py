"""The NTT pass geometry of csrc/mlpcs.hip restated on the CPU: ntt_plan's
stage ranges and tiles, the radix-2 pass (k_ntt_pass) and the radix-4 pass
(k_ntt_pass4: two stages per LDS round trip, three twiddles per group of four,
an odd leftover stage as radix-2) with exact integers.  DIF takes natural
order to bit-reversed, DIT bit-reversed to natural; forward then inverse must
give n a, and DIF outputs must equal the DFT."""
import random

import pytest

import quill_oracle as o
R=o.R_MOD
NTT_LGT=11
def plan(logn, T=NTT_LGT):
    v=[];s=0
    while s<logn:
        B=min(T if s==0 else 7, logn-s)
        lgL=min(T-B, s); lgL=min(lgL, logn-B)
        v.append((s,B,lgL)); s+=B
    return v
def run_pass(a, tw, logn, s0, B, lgL, DIF, r4):
    n=len(a); lgT=B+lgL; T=1<<lgT; L=1<<lgL
    ngroups=(1<<s0)>>lgL
    out=a[:]
    for blk in range(n>>lgT):
        hi=blk//ngroups; lo0=(blk%ngroups)<<lgL
        base=(hi<<(s0+B))+lo0
        idx=[base+((e>>lgL)<<s0)+(e&(L-1)) for e in range(T)]
        sh=[a[i] for i in idx]
        def r2(b):
            s=s0+b
            for p in range(T//2):
                l=p&(L-1); q=p>>lgL
                mid0=((q>>b)<<(b+1))|(q&((1<<b)-1))
                e0=(mid0<<lgL)|l; e1=e0|(1<<(b+lgL))
                j=((mid0&((1<<b)-1))<<s0)+lo0+l
                w=tw[j<<(logn-1-s)]
                u,v=sh[e0],sh[e1]
                if DIF: sh[e0]=(u+v)%R; sh[e1]=(u-v)*w%R
                else: t=v*w%R; sh[e0]=(u+t)%R; sh[e1]=(u-t)%R
        def rr4(b):
            bl=b-1 if DIF else b
            for g in range(T//4):
                l=g&(L-1); q=g>>lgL
                mid0=((q>>bl)<<(bl+2))|(q&((1<<bl)-1))
                e00=(mid0<<lgL)|l; dl=1<<(bl+lgL); dh=2<<(bl+lgL)
                e=[e00,e00|dl,e00|dh,e00|dl|dh]
                j0=((mid0&((1<<bl)-1))<<s0)+lo0+l; sl=s0+bl
                wa=tw[j0<<(logn-2-sl)]; wb=tw[(j0+(1<<sl))<<(logn-2-sl)]; wc=tw[j0<<(logn-1-sl)]
                x=[sh[k] for k in e]
                if DIF:
                    x0,x1,x2,x3=x
                    x0,x2=(x0+x2)%R,(x0-x2)*wa%R
                    x1,x3=(x1+x3)%R,(x1-x3)*wb%R
                    x0,x1=(x0+x1)%R,(x0-x1)*wc%R
                    x2,x3=(x2+x3)%R,(x2-x3)*wc%R
                else:
                    x0,x1,x2,x3=x
                    t1=x1*wc%R; x0,x1=(x0+t1)%R,(x0-t1)%R
                    t3=x3*wc%R; x2,x3=(x2+t3)%R,(x2-t3)%R
                    t2=x2*wa%R; x0,x2=(x0+t2)%R,(x0-t2)%R
                    t3=x3*wb%R; x1,x3=(x1+t3)%R,(x1-t3)%R
                for k,v in zip(e,[x0,x1,x2,x3]): sh[k]=v
        if not r4:
            for k in range(B):
                r2(B-1-k if DIF else k)
        elif DIF:
            b=B-1
            if B&1: r2(b); b-=1
            while b>=1: rr4(b); b-=2
        else:
            b=0
            while b+1<B: rr4(b); b+=2
            if b<B: r2(b)
        for e,i in enumerate(idx): out[i]=sh[e]
    return out
def ntt(a, logn, DIF, r4):
    w=o.two_adic_root(logn) if DIF else o.fr_inv(o.two_adic_root(logn))
    n=1<<logn; tw=[pow(w,k,R) for k in range(n//2)]
    P=plan(logn)
    if DIF: P=P[::-1]
    for (s0,B,lgL) in P:
        use4 = r4 and B+lgL==NTT_LGT and B>=2
        a=run_pass(a,tw,logn,s0,B,lgL,DIF,use4)
    return a


def bitrev(x, b):
    return int(format(x, f"0{b}b")[::-1], 2) if b else 0


@pytest.mark.parametrize("logn", [3, 11, 12, 13, 15])
@pytest.mark.parametrize("r4", [False, True])
def test_ntt_passes_roundtrip(logn, r4):
    n = 1 << logn
    rnd = random.Random(logn)
    a = [rnd.randrange(R) for _ in range(n)]
    F = ntt(a, logn, True, r4)
    w = o.two_adic_root(logn)
    for k in [0, 1, 5, n - 1, n // 3]:
        if n <= 4096:
            assert F[bitrev(k, logn)] == sum(a[j] * pow(w, j * k, R) for j in range(n)) % R
    A = ntt(F, logn, False, r4)
    assert A == [x * n % R for x in a]
