"""The NTT pass geometry of csrc/mlpcs.hip restated on the CPU: ntt_plan's
stage ranges and tiles, the radix-2 pass k_ntt_pass with its twiddles read
from the stage pyramid (k_tw_pyramid: pyr[2^s - 1 + j] = w^(j 2^(logn-1-s)))
or the flat table, and a radix-4 variant (two stages per LDS round trip,
three twiddles per group of four; measured no faster on MI355X, not in the
library) with exact integers.  DIF takes natural order to bit-reversed, DIT
bit-reversed to natural; forward then inverse must give n a, and DIF outputs
must equal the DFT."""
import random

import pytest

import quill_oracle as o

R = o.R_MOD
NTT_LGT = 10  # log2 of the 1024-element LDS tile


def ntt_plan(logn):
    """[(s0, B, lgL)]: stages [s0, s0 + B) on tiles of 2^B mid x 2^lgL lo indices"""
    v, s = [], 0
    while s < logn:
        B = min(NTT_LGT if s == 0 else 7, logn - s)
        lgL = min(NTT_LGT - B, s, logn - B)
        v.append((s, B, lgL))
        s += B
    return v


def twiddle(tw, pyr, logn, s, j):
    """k_ntt_pass's twiddle load: pyramid entry 2^s - 1 + j or flat j 2^(logn-1-s)"""
    return pyr[(1 << s) - 1 + j] if pyr is not None else tw[j << (logn - 1 - s)]


def pyramid(tw, logn):
    """k_tw_pyramid"""
    out = []
    for i in range((1 << logn) - 1):
        st = (i + 1).bit_length() - 1
        out.append(tw[(i + 1 - (1 << st)) << (logn - 1 - st)])
    return out


def run_pass(a, tw, logn, s0, B, lgL, dif, radix4, pyr=None):
    n, T, L = len(a), 1 << (B + lgL), 1 << lgL
    ngroups = (1 << s0) >> lgL
    out = a[:]
    for blk in range(n >> (B + lgL)):
        hi, lo0 = blk // ngroups, (blk % ngroups) << lgL
        base = (hi << (s0 + B)) + lo0
        idx = [base + ((e >> lgL) << s0) + (e & (L - 1)) for e in range(T)]
        sh = [a[i] for i in idx]

        def radix2(b):
            s = s0 + b
            for p in range(T // 2):
                l, q = p & (L - 1), p >> lgL
                mid0 = ((q >> b) << (b + 1)) | (q & ((1 << b) - 1))
                e0 = (mid0 << lgL) | l
                e1 = e0 | (1 << (b + lgL))
                w = twiddle(tw, pyr, logn, s, ((mid0 & ((1 << b) - 1)) << s0) + lo0 + l)
                u, v = sh[e0], sh[e1]
                if dif:
                    sh[e0], sh[e1] = (u + v) % R, (u - v) * w % R
                else:
                    t = v * w % R
                    sh[e0], sh[e1] = (u + t) % R, (u - t) % R

        def radix4(b):
            bl = b - 1 if dif else b  # the lower of the two stage bits
            for g in range(T // 4):
                l, q = g & (L - 1), g >> lgL
                mid0 = ((q >> bl) << (bl + 2)) | (q & ((1 << bl) - 1))
                e00 = (mid0 << lgL) | l
                dl, dh = 1 << (bl + lgL), 2 << (bl + lgL)
                e = [e00, e00 | dl, e00 | dh, e00 | dl | dh]
                j0 = ((mid0 & ((1 << bl) - 1)) << s0) + lo0 + l
                sl = s0 + bl
                wa = tw[j0 << (logn - 2 - sl)]
                wb = tw[(j0 + (1 << sl)) << (logn - 2 - sl)]
                wc = tw[j0 << (logn - 1 - sl)]
                x0, x1, x2, x3 = (sh[k] for k in e)
                if dif:
                    x0, x2 = (x0 + x2) % R, (x0 - x2) * wa % R
                    x1, x3 = (x1 + x3) % R, (x1 - x3) * wb % R
                    x0, x1 = (x0 + x1) % R, (x0 - x1) * wc % R
                    x2, x3 = (x2 + x3) % R, (x2 - x3) * wc % R
                else:
                    t1, t3 = x1 * wc % R, x3 * wc % R
                    x0, x1 = (x0 + t1) % R, (x0 - t1) % R
                    x2, x3 = (x2 + t3) % R, (x2 - t3) % R
                    t2, t3 = x2 * wa % R, x3 * wb % R
                    x0, x2 = (x0 + t2) % R, (x0 - t2) % R
                    x1, x3 = (x1 + t3) % R, (x1 - t3) % R
                for k, v in zip(e, (x0, x1, x2, x3)):
                    sh[k] = v

        if not radix4:
            for k in range(B):
                radix2(B - 1 - k if dif else k)
        elif dif:
            b = B - 1
            if B & 1:
                radix2(b)
                b -= 1
            while b >= 1:
                radix4(b)
                b -= 2
        else:
            b = 0
            while b + 1 < B:
                radix4(b)
                b += 2
            if b < B:
                radix2(b)
        for e, i in enumerate(idx):
            out[i] = sh[e]
    return out


def ntt(a, logn, dif, radix4, use_pyr=True):
    """ntt_run: twiddles w^k (k < n/2), passes in plan order (reversed for DIF);
    the radix-4 variant takes full tiles with at least two stages"""
    w = o.two_adic_root(logn) if dif else o.fr_inv(o.two_adic_root(logn))
    tw = [pow(w, k, R) for k in range((1 << logn) // 2)]
    pyr = pyramid(tw, logn) if use_pyr else None
    plan = ntt_plan(logn)
    for s0, B, lgL in (plan[::-1] if dif else plan):
        a = run_pass(a, tw, logn, s0, B, lgL, dif, radix4 and B + lgL == NTT_LGT and B >= 2, pyr)
    return a


def bitrev(x, b):
    return int(format(x, f"0{b}b")[::-1], 2) if b else 0


@pytest.mark.parametrize("logn", [3, 10, 11, 12, 13, 15])
@pytest.mark.parametrize("radix4,use_pyr", [(False, True), (False, False), (True, True)])
def test_ntt_passes_roundtrip(logn, radix4, use_pyr):
    n = 1 << logn
    rnd = random.Random(logn)
    a = [rnd.randrange(R) for _ in range(n)]
    F = ntt(a, logn, True, radix4, use_pyr)
    w = o.two_adic_root(logn)
    if n <= 4096:
        for k in [0, 1, 5, n - 1, n // 3]:
            assert F[bitrev(k, logn)] == sum(a[j] * pow(w, j * k, R) for j in range(n)) % R
    assert ntt(F, logn, False, radix4, use_pyr) == [x * n % R for x in a]


def test_plan_tiles():
    assert ntt_plan(10) == [(0, 10, 0)]
    assert ntt_plan(11) == [(0, 10, 0), (10, 1, 9)]
    assert ntt_plan(24) == [(0, 10, 0), (10, 7, 3), (17, 7, 3)]


@pytest.mark.parametrize("logn", [1, 2, 5, 9])
def test_eqdft_bitrev_twiddle_index(logn):
    """k_eqdft_level reads twb[k >> 1] (twb = flat table in bit-reversed order),
    negated for odd k, where the product formula needs w^(bitrev_{L-t}(k) 2^t)
    (csrc/mlpcs.hip): the same exponent for every level t and entry k."""
    half = 1 << (logn - 1)
    twb = [bitrev(i, logn - 1) for i in range(half)]  # exponents held by twb
    for t in range(logn):
        for k in range(1 << (logn - t)):
            m = bitrev(k, logn - t) << t
            assert twb[k >> 1] == m & (half - 1)
            assert ((m & half) != 0) == bool(k & 1)


@pytest.mark.parametrize("lb", [1, 2, 6, 9])
def test_combine_res_bitrev_twiddle_index(lb):
    """k_s_combine_res reads twiBb[p >> 1] (bit-reversed w_B^{-e} table) with
    the sign from p's low bit and the `alt` flip from p's top bit, where the
    combine needs w_B^{-k2}, k2 = bitrev_lb(p), reduced by w_B^{B/2} = -1."""
    half = 1 << (lb - 1)
    twb = [bitrev(i, lb - 1) for i in range(half)]
    for p in range(1 << lb):
        k2 = bitrev(p, lb)
        assert twb[p >> 1] == k2 & (half - 1)
        assert ((k2 & half) != 0) == bool(p & 1)
        assert bool(k2 & 1) == bool((p >> (lb - 1)) & 1)


M29 = (1 << 29) - 1
P_FR = R


def _limbs29(x):
    return [(x >> (29 * i)) & (M29 if i < 8 else 0xffffffff) for i in range(9)]


def _redundant(kp):
    """field29.h l9_redundant: limbs 0..7 raised by 2^29 (borrowed from above)"""
    r = list(kp)
    r[0] += 1 << 29
    for i in range(1, 8):
        r[i] += (1 << 29) - 1
    r[8] -= 1
    return r


def _val(limbs):
    return sum(l << (29 * i) for i, l in enumerate(limbs))


@pytest.mark.parametrize("seed", range(4))
def test_dit_butterfly_sub_2p_redundant(seed):
    """k_ntt_pass DIT: v' = red2p29(subk29(u, t, K2)) with K2 = 2p in redundant
    limbs, u, t < 2p normalized (csrc/field29.h).  Restated limb by limb in
    uint32 arithmetic: the top limb may wrap below zero, normfull29's carry
    brings it back (the value u + 2p - t is >= 0), one conditional subtraction
    of 2p leaves [0, 2p) - equal to (u - t) mod p."""
    rnd = random.Random(seed)
    K2 = _redundant(_limbs29(2 * P_FR))
    edge = [0, 1, P_FR - 1, P_FR, 2 * P_FR - 1]
    cases = [(a, b) for a in edge for b in edge] + \
            [(rnd.randrange(2 * P_FR), rnd.randrange(2 * P_FR)) for _ in range(2000)]
    for u, t in cases:
        ul, tl = _limbs29(u), _limbs29(t)
        a = [(ul[i] + (K2[i] - tl[i])) & 0xffffffff for i in range(9)]
        c, r = 0, []
        for i in range(8):  # normfull29
            x = (a[i] + c) & 0xffffffff
            r.append(x & M29)
            c = x >> 29
        r.append((a[8] + c) & 0xffffffff)
        v = _val(r)
        assert 0 <= v < 4 * P_FR
        v = v - 2 * P_FR if v >= 2 * P_FR else v  # condsub29(., 2p)
        assert v < 2 * P_FR and v % P_FR == (u - t) % P_FR
