"""The residue-split S polynomial (csrc/mlpcs.hip s_poly_sharded) restated step
for step on the CPU, W ranks simulated in-process, against the oracle's
compute_s_polynomial (ipa.rs:122-157): the forward pre-sum per residue, the
B-point DIF with bit-reversed output, G at the residue from the eq product
formula restricted to the residue (k_eqdft_res: host-collapsed top levels,
then one level per launch in bit-reversed order), the combine with the mirror
residue (k_s_combine_res), the B-point inverse, the pre-multiplied outgoing
vectors (k_s_outgoing) and the all-to-all + sum (k_s_sum_parts).  Naive DFTs
stand in for the device NTT passes (same transform, same output order)."""
import random

import pytest

import quill_oracle as o

R = o.R_MOD


def bitrev(x, bits):
    return int(format(x, f"0{bits}b")[::-1], 2) if bits else 0


def dft(a, w):
    n = len(a)
    return [sum(a[j] * pow(w, j * k, R) for j in range(n)) % R for k in range(n)]


def rank_slice(f, point, W, c):
    """this rank's outgoing vectors send[d][m] (d < W, m < L)"""
    M = len(f)
    nvars = len(point)
    n, L = 2 * M, M // W
    B = 2 * L
    lb = B.bit_length() - 1
    w = o.two_adic_root(n.bit_length() - 1)
    wi = o.fr_inv(w)
    wB = pow(w, W, R)
    wW = pow(w, B, R)
    ninv = o.fr_inv(n)
    cm = (W - c) % W
    FG = {}
    for cc in sorted({c, cm}):
        # u_cc[i2] = w^{i2 cc} sum_{i1 < W/2} w_W^{i1 cc} f[i1 B + i2]
        # (W = 1: one block, f fills its first half; the rest is zero padding)
        u = [pow(w, i2 * cc, R) * sum(pow(wW, i1 * cc, R) * f[i1 * B + i2]
                                      for i1 in range(max(W // 2, 1)) if i1 * B + i2 < M)
             % R for i2 in range(B)]
        Fnat = dft(u, wB)  # F[k2 W + cc], natural k2
        Fbr = [Fnat[bitrev(p, lb)] for p in range(B)]
        # G: levels t >= lb collapse to q0; levels lb-1 .. 0 in bit-reversed order
        q0 = 1
        for t in range(nvars - 1, lb - 1, -1):
            zt = point[t]
            q0 = q0 * ((1 - zt) + zt * pow(w, cc << t, R)) % R
        prev = None
        for t in range(min(nvars, lb) - 1, -1, -1):  # W = 1: nvars = lb - 1
            bits = lb - t
            zt = point[t]
            cur = []
            for e in range(1 << bits):
                k2 = bitrev(e, bits)
                fct = ((1 - zt) + zt * pow(w, cc << t, R) * pow(wB, k2 << t, R)) % R
                cur.append(fct * (q0 if prev is None else prev[e >> 1]) % R)
            prev = cur
        FG[cc] = (Fbr, prev)
    Fc, Gc = FG[c]
    Fm, Gm = FG[cm]
    cst = pow(wi, c, R) * ninv % R
    if c & 1:
        cst = (-cst) % R
    H = []
    for p in range(B):
        if c:
            pp = ~p & (B - 1)
        else:
            pp = p ^ ((1 << (p.bit_length() - 1)) - 1) if p else 0
        k2 = bitrev(p, lb)
        v = (Fc[p] * Gm[pp] + Fm[pp] * Gc[p]) % R
        # w^{k(M-1)} = (-1)^k w^{-k}, k = k2 W + c: (-1)^k = (-1)^c for even W,
        # (-1)^k2 at W = 1
        sgn = -1 if (W == 1 and k2 & 1) else 1
        H.append(sgn * v * pow(wB, -k2 % B, R) % R * cst % R)
    # inverse DIT: bit-reversed in, natural out: Z[i2] = sum_k2 H[bitrev(k2)] wB^{-i2 k2}
    Hnat = [H[bitrev(k2, lb)] for k2 in range(B)]
    Z = dft(Hnat, o.fr_inv(wB))
    out = []
    for d in range(W):
        # S[d L + m] = h[M + d L + m] = h[i1 B + i2]: i1 = W/2 + d/2 and
        # i2 = (d mod 2) L + m for W >= 2; i1 = 0, i2 = L + m at W = 1
        i1, o2 = divmod(M + d * L, B)
        K = pow(o.fr_inv(wW), (i1 * c) % W, R)
        out.append([K * pow(wi, c * (o2 + m), R) % R * Z[o2 + m] % R for m in range(L)])
    return out


@pytest.mark.parametrize("nvars,W", [(3, 2), (4, 4), (4, 8), (5, 2), (5, 8), (6, 4), (3, 1), (5, 1)])
def test_residue_split_s_polynomial(nvars, W):
    rnd = random.Random(nvars * 10 + W)
    M = 1 << nvars
    f = [rnd.randrange(R) for _ in range(M)]
    point = [rnd.randrange(R) for _ in range(nvars)]
    g = o.fast_eq_eval_hypercube(nvars, point)
    S = o.compute_s_polynomial(f, g)
    S = S + [0] * (M - len(S))  # untrimmed, plus h[2M - 1] = 0
    sends = [rank_slice(f, point, W, c) for c in range(W)]
    L = M // W
    for d in range(W):  # all-to-all, then the sum on rank d
        got = [sum(sends[s][d][m] for s in range(W)) % R for m in range(L)]
        assert got == S[d * L:(d + 1) * L], (d, W)


def test_half_size_inverse_identity():
    """The half-size inverse of s_poly_device (k_s_combine_half, k_sym_*,
    round 6), restated on the CPU: with P_j = F_j G_-j + F_-j G_j (even), D_j =
    (P_j + P_{j+N2}) + (P_j - P_{j+N2}) w^-j, d = IDFT_N2(D), b_e = b_0 +
    sum_{t<=e} (d_t - d_{N2-t}) with b_0 = sum_j B_j, a = d - b: S_{2e-1} = a_e
    / n and S_{2e} = b_e / n equal compute_s_polynomial (ipa.rs:122-157) for
    even, odd, power-of-two and ragged lengths (n = 2^ceil(log2(2M - 1)))."""
    import random
    rnd = random.Random(66)
    R = o.R_MOD

    def dft(a, w):
        return [sum(a[i] * pow(w, i * j, R) for i in range(len(a))) % R for j in range(len(a))]
    for M in (2, 3, 5, 8, 13, 16, 21):
        f = [rnd.randrange(R) for _ in range(M)]
        g = [rnd.randrange(R) for _ in range(rnd.randrange(1, M + 1))]
        S = o.compute_s_polynomial(f, g)
        S = S + [0] * (M - 1 - len(S))
        logn = 1
        while (1 << logn) < 2 * M - 1:
            logn += 1
        n, N2 = 1 << logn, 1 << (logn - 1)
        w = o.two_adic_root(logn)
        wi = pow(w, R - 2, R)
        F = dft(f + [0] * (n - M), w)
        G = dft(g + [0] * (n - len(g)), w)
        P = [(F[j] * G[-j % n] + F[-j % n] * G[j]) % R for j in range(n)]
        ninv = pow(n, R - 2, R)
        B = [(P[j] - P[j + N2]) * pow(wi, j, R) % R for j in range(N2)]
        D = [(P[j] + P[j + N2] + B[j]) * ninv % R for j in range(N2)]
        d = dft(D, wi * wi % R)
        b = [sum(B) * ninv % R]
        for e in range(1, (M - 1) // 2 + 1):
            b.append((b[-1] + d[e] - d[N2 - e]) % R)
        out = [None] * (M - 1)
        for e, be in enumerate(b):
            if 2 * e + 2 <= M:
                out[2 * e] = be
            if e >= 1 and 2 * e + 1 <= M:
                out[2 * e - 1] = (d[e] - be) % R
        assert out == S, M
