"""CPU restatement of the Quill prover hot path — TEST INFRASTRUCTURE ONLY.

This module is the *oracle* (checker).  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker —
never as the thing measured or shipped.  The product path lives in
``quill-zkvm_amd/`` (HIP kernels behind the C-ABI in ``include/quill_gpu.h``) and
fails loudly when its shared library is missing.

Pinning.  The reference (Rust + arkworks 0.5.0 + blake3 1.8.2) cannot be compiled
or imported in this container (no cargo/rustc, crates not vendored; see
DESIGN.md "Oracle").  This restatement is pinned by
  * every known-answer test the reference's own tests hold
    (pcs/src/ipa.rs:230,273; pcs/src/mlpcs.rs:226-242,283-285,423-429;
    hyperplonk/src/utils/eq_eval.rs:61-74; hyperplonk/src/piops/sumcheck.rs:216-228;
    hyperplonk/src/piops/zerocheck.rs:142-158) — see tests/test_oracle_kats.py;
  * the BLAKE3 specification's published digests (blake3_py.py);
  * mathematical identities (commit == [p(tau)]G for a known-tau SRS; the unique
    group element an MSM denotes; p(0)+p(1) = claim for sumcheck rounds).
Transcript *bytes* (ark-serialize encodings) are "parity unpinned" by reference
tests: no reference test asserts hash or serialization bytes; the encodings
follow ark-serialize 0.5.0 as documented in SURVEY.md §8(c).

All arithmetic is exact Python-int modular arithmetic (no floating point).
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from blake3_py import blake3, blake3_xof  # noqa: E402

# ---------------------------------------------------------------------------
# BN254 parameters (ark-bn254 0.5.0, Cargo.lock:24-25)
# ---------------------------------------------------------------------------
R_MOD = 21888242871839275222246405745257275088548364400416034343698204186575808495617
P_MOD = 21888242871839275222246405745257275088696311157297823662689037894645226208583
FR_BITS = 254
TWO_ADICITY = 28
FR_GENERATOR = 5  # ark-bn254 Fr multiplicative generator
G1_B = 3  # y^2 = x^3 + 3
G1_GEN = (1, 2)  # ark-bn254 G1 generator (affine)
MONT_R = 1 << 256  # arkworks Montgomery radix for 4x64-bit limbs


def fr(x) -> int:
    return x % R_MOD


def fr_inv(x: int) -> int:
    x %= R_MOD
    if x == 0:
        raise ZeroDivisionError("inverse of zero in Fr")
    return pow(x, R_MOD - 2, R_MOD)


def fq_inv(x: int) -> int:
    x %= P_MOD
    if x == 0:
        raise ZeroDivisionError("inverse of zero in Fq")
    return pow(x, P_MOD - 2, P_MOD)


def to_mont(x: int, mod: int = R_MOD) -> int:
    return (x * MONT_R) % mod


def from_mont(x: int, mod: int = R_MOD) -> int:
    return (x * pow(MONT_R, -1, mod)) % mod


# ---------------------------------------------------------------------------
# G1 arithmetic (affine tuples; None = point at infinity)
# ---------------------------------------------------------------------------
def g1_is_on_curve(P) -> bool:
    if P is None:
        return True
    x, y = P
    return (y * y - x * x * x - G1_B) % P_MOD == 0


def g1_neg(P):
    if P is None:
        return None
    return (P[0], (-P[1]) % P_MOD)


def _jac_double(X, Y, Z):
    if Z == 0 or Y == 0:
        return (0, 1, 0)
    p = P_MOD
    A = X * X % p
    B = Y * Y % p
    C = B * B % p
    D = 2 * ((X + B) * (X + B) - A - C) % p
    E = 3 * A % p
    F = E * E % p
    X3 = (F - 2 * D) % p
    Y3 = (E * (D - X3) - 8 * C) % p
    Z3 = 2 * Y * Z % p
    return (X3, Y3, Z3)


def _jac_add(P1, P2):
    X1, Y1, Z1 = P1
    X2, Y2, Z2 = P2
    if Z1 == 0:
        return P2
    if Z2 == 0:
        return P1
    p = P_MOD
    Z1Z1 = Z1 * Z1 % p
    Z2Z2 = Z2 * Z2 % p
    U1 = X1 * Z2Z2 % p
    U2 = X2 * Z1Z1 % p
    S1 = Y1 * Z2 * Z2Z2 % p
    S2 = Y2 * Z1 * Z1Z1 % p
    if U1 == U2:
        if S1 == S2:
            return _jac_double(X1, Y1, Z1)
        return (0, 1, 0)
    H = (U2 - U1) % p
    I = (2 * H) * (2 * H) % p
    J = H * I % p
    r = 2 * (S2 - S1) % p
    V = U1 * I % p
    X3 = (r * r - J - 2 * V) % p
    Y3 = (r * (V - X3) - 2 * S1 * J) % p
    Z3 = ((Z1 + Z2) * (Z1 + Z2) - Z1Z1 - Z2Z2) * H % p
    return (X3, Y3, Z3)


def _to_jac(P):
    return (0, 1, 0) if P is None else (P[0], P[1], 1)


def _from_jac(J):
    X, Y, Z = J
    if Z % P_MOD == 0:
        return None
    zi = fq_inv(Z)
    zi2 = zi * zi % P_MOD
    return (X * zi2 % P_MOD, Y * zi2 * zi % P_MOD)


def g1_add(P, Q):
    return _from_jac(_jac_add(_to_jac(P), _to_jac(Q)))


def g1_mul(P, k: int):
    """[k]P by double-and-add (k taken mod r: G1 has prime order r)."""
    k %= R_MOD
    acc = (0, 1, 0)
    base = _to_jac(P)
    while k:
        if k & 1:
            acc = _jac_add(acc, base)
        base = _jac_double(*base)
        k >>= 1
    return _from_jac(acc)


def g1_msm_naive(bases, scalars):
    """Sum_i scalars[i]*bases[i] over min(len) terms.

    Semantics of ark-ec `VariableBaseMSM::msm_unchecked` as called at
    pcs/src/kzg.rs:72 (truncates to the shorter input)."""
    acc = (0, 1, 0)
    for P, s in zip(bases, scalars):
        s %= R_MOD
        if s == 0 or P is None:
            continue
        acc = _jac_add(acc, _to_jac(g1_mul(P, s)))
    return _from_jac(acc)


# ---------------------------------------------------------------------------
# ark-serialize 0.5.0 uncompressed encodings (parity unpinned)
# ---------------------------------------------------------------------------
def ser_u64(v: int) -> bytes:
    """`usize` / `u64` -> 8 bytes LE (transcript absorbs `num_vars: usize`,
    hyperplonk/src/piops/sumcheck.rs:35)."""
    return int(v).to_bytes(8, "little")


def ser_fr(x: int) -> bytes:
    """Fr -> 32 bytes canonical little-endian (serialize_with_flags, EmptyFlags)."""
    return (x % R_MOD).to_bytes(32, "little")


def ser_fr_vec(xs) -> bytes:
    """`Vec<F>` / `&[F]` -> u64 LE length prefix + items."""
    return ser_u64(len(xs)) + b"".join(ser_fr(x) for x in xs)


def poly_trim(coeffs):
    """ark-poly DensePolynomial::truncate_leading_zeros (trailing in LE order)."""
    c = [x % R_MOD for x in coeffs]
    while c and c[-1] == 0:
        c.pop()
    return c


def ser_poly(coeffs) -> bytes:
    """DensePolynomial (derived CanonicalSerialize of `coeffs: Vec<F>`), trimmed."""
    return ser_fr_vec(poly_trim(coeffs))


def ser_g1(P) -> bytes:
    """G1 projective/affine uncompressed: x (32 B LE) || y (32 B LE) with the SW
    flags in the top two bits of y's last byte: bit7 = y is "negative"
    (y > p - y), bit6 = infinity (x = y = 0)."""
    if P is None:
        out = bytearray(64)
        out[63] |= 0x40
        return bytes(out)
    x, y = P
    out = bytearray(x.to_bytes(32, "little") + y.to_bytes(32, "little"))
    if y > P_MOD - y:
        out[63] |= 0x80
    return bytes(out)


def de_g1(b: bytes):
    if b[63] & 0x40:
        return None
    yb = bytearray(b[32:64])
    yb[31] &= 0x3F
    return (int.from_bytes(b[:32], "little"), int.from_bytes(bytes(yb), "little"))


# ---------------------------------------------------------------------------
# Transcript (transcript/src/transcript.rs:5-74)
# ---------------------------------------------------------------------------
class Transcript:
    """BLAKE3 hash-chain Fiat-Shamir transcript.

    new:    state = B3(domain)                               transcript.rs:14-22
    append: state = B3(state || msg)                         transcript.rs:25-31
    draw:   out = B3-XOF(state || "challenge")[0..n]; append(out)   :48-62
    Fr:     LE(48 bytes) mod r  ((254+128+7)/8 = 48)          :70-74
    """

    def __init__(self, domain: bytes):
        self.domain = bytes(domain)
        self.state = blake3(self.domain)

    def append_bytes(self, msg: bytes):
        self.state = blake3(self.state + bytes(msg))

    def append_u64(self, v: int):
        self.append_bytes(ser_u64(v))

    def append_fr(self, x: int):
        self.append_bytes(ser_fr(x))

    def append_fr_vec(self, xs):
        self.append_bytes(ser_fr_vec(xs))

    def append_poly(self, coeffs):
        self.append_bytes(ser_poly(coeffs))

    def append_g1(self, P):
        self.append_bytes(ser_g1(P))

    def draw_challenge(self, n: int) -> bytes:
        out = blake3_xof(self.state + b"challenge", n)
        self.append_bytes(out)
        return out

    def draw_field_element(self) -> int:
        nbytes = (FR_BITS + 128 + 7) // 8
        return int.from_bytes(self.draw_challenge(nbytes), "little") % R_MOD

    def clone(self) -> "Transcript":
        t = Transcript.__new__(Transcript)
        t.domain, t.state = self.domain, self.state
        return t


# ---------------------------------------------------------------------------
# Univariate polynomial helpers (ark-poly DensePolynomial semantics)
# ---------------------------------------------------------------------------
def poly_add(a, b):
    n = max(len(a), len(b))
    return poly_trim([(a[i] if i < len(a) else 0) + (b[i] if i < len(b) else 0)
                      for i in range(n)])


def poly_mul(a, b):
    a, b = poly_trim(a), poly_trim(b)
    if not a or not b:
        return []
    out = [0] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        if x == 0:
            continue
        for j, y in enumerate(b):
            out[i + j] += x * y
    return poly_trim(out)


def poly_eval(coeffs, x: int) -> int:
    """Horner (ark-poly `Polynomial::evaluate`), kzg.rs:77-78."""
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % R_MOD
    return acc


def poly_div_linear(coeffs, x: int):
    """q = (p - p(x)) / (X - x) by synthetic division; returns (q, y).

    Same quotient as kzg.rs:81-84 (`&numerator / &denominator`), trimmed."""
    c = poly_trim(coeffs)
    if not c:
        return [], 0
    n = len(c)
    q = [0] * (n - 1)
    acc = 0
    for i in range(n - 1, 0, -1):
        acc = (acc * x + c[i]) % R_MOD
        q[i - 1] = acc
    y = (acc * x + c[0]) % R_MOD
    return poly_trim(q), y


# ---------------------------------------------------------------------------
# Radix-2 FFT over Fr (ark-poly Radix2EvaluationDomain semantics)
# ---------------------------------------------------------------------------
def two_adic_root(log_n: int) -> int:
    """Primitive 2^log_n-th root of unity (subgroup is unique; interpolation
    results do not depend on which generator is used)."""
    assert log_n <= TWO_ADICITY
    w = pow(FR_GENERATOR, (R_MOD - 1) >> TWO_ADICITY, R_MOD)
    return pow(w, 1 << (TWO_ADICITY - log_n), R_MOD)


def ntt(a, inverse=False):
    n = len(a)
    log_n = n.bit_length() - 1
    assert 1 << log_n == n
    w = two_adic_root(log_n)
    if inverse:
        w = fr_inv(w)
    out = [0] * n
    for k in range(n):
        s = 0
        wk = pow(w, k, R_MOD)
        acc = 1
        for j in range(n):
            s += a[j] * acc
            acc = acc * wk % R_MOD
        out[k] = s % R_MOD
    if inverse:
        ninv = fr_inv(n)
        out = [x * ninv % R_MOD for x in out]
    return out


# ---------------------------------------------------------------------------
# eq tables (hyperplonk/src/utils/eq_eval.rs)
# ---------------------------------------------------------------------------
def fast_eq_eval_hypercube(n: int, point):
    """eq(bin(i), point) for i in [0, 2^n); bit j of i <-> point[j].

    Restates eq_eval.rs:6-31: iterate i = n-1 .. 0, eval -> (eval*(1-r_i), eval*r_i)."""
    assert len(point) == n
    evals = [1]
    for i in reversed(range(n)):
        r = point[i] % R_MOD
        omr = (1 - r) % R_MOD
        new = []
        for e in evals:
            new.append(e * omr % R_MOD)
            new.append(e * r % R_MOD)
        evals = new
    assert len(evals) == 1 << n
    return evals


def eq_eval(x, r) -> int:
    """eq_eval.rs:33-43."""
    assert len(x) == len(r)
    res = 1
    for xi, ri in zip(x, r):
        res = res * (xi * ri + (1 - xi) * (1 - ri)) % R_MOD
    return res


# ---------------------------------------------------------------------------
# KZG (pcs/src/kzg.rs) with a known-tau SRS
# ---------------------------------------------------------------------------
class KZG:
    """KZG over BN254 G1 with an explicit (seeded) tau.

    g1_points[i] = [tau^i] g1 (kzg.rs:35-59).  `verify` uses the trapdoor
    identity C - [y]g1 == [tau - x] pi (equivalent to the pairing check at
    kzg.rs:98-108 for a known tau; no pairing is implemented here)."""

    def __init__(self, max_degree: int, tau: int, g1=G1_GEN, points=None):
        self.max_degree = max_degree
        self.tau = tau % R_MOD
        self.g1 = g1
        self._taus = None
        self._points = points

    @property
    def taus(self):
        if self._taus is None:
            self._taus = [pow(self.tau, i, R_MOD) for i in range(self.max_degree + 1)]
        return self._taus

    @property
    def g1_points(self):
        if self._points is None:
            self._points = [g1_mul(self.g1, t) for t in self.taus]
        return self._points

    def commit(self, poly):
        """kzg.rs:61-73 — Sum poly[i] * g1_points[i] (length <= max_degree+1).

        Evaluated through the trapdoor: the MSM denotes [p(tau)] g1, a unique
        group element; `commit_msm` runs the literal MSM for small sizes."""
        assert len(poly) <= self.max_degree + 1, "Polynomial degree exceeds max degree"
        return g1_mul(self.g1, poly_eval(poly, self.tau))

    def commit_msm(self, poly):
        assert len(poly) <= self.max_degree + 1
        return g1_msm_naive(self.g1_points, poly)

    def open(self, poly, x):
        """kzg.rs:75-96 -> (x, y, pi)."""
        q, y = poly_div_linear(poly, x % R_MOD)
        # kzg.rs:85 sanity: q*(X-x) == p - y
        assert poly_mul(q, [(-x) % R_MOD, 1]) == poly_add(poly, [(-y) % R_MOD]), \
            "Polynomial division failed"
        return (x % R_MOD, y, self.commit(q))

    def verify(self, C, proof) -> bool:
        x, y, pi = proof
        lhs = g1_add(C, g1_neg(g1_mul(self.g1, y)))
        rhs = g1_mul(pi, (self.tau - x) % R_MOD)
        return lhs == rhs


# ---------------------------------------------------------------------------
# Inner-product / multilinear PCS (pcs/src/ipa.rs, pcs/src/mlpcs.rs)
# ---------------------------------------------------------------------------
def compute_s_polynomial(f, g):
    """ipa.rs:122-157: pad to M = max len, h = f*rev(g) + rev(f)*g,
    pad h to 2M-1, S = h[(2M-1)//2 + 1 ..], trimmed."""
    M = max(len(f), len(g))
    f = list(f) + [0] * (M - len(f))
    g = list(g) + [0] * (M - len(g))
    h = poly_add(poly_mul(f, g[::-1]), poly_mul(f[::-1], g))
    h = h + [0] * (2 * M - 1 - len(h))
    return poly_trim(h[(len(h) // 2 + 1):])


def compute_s_polynomial_corr(f, g):
    """Equivalent closed form S_k = sum_i (f_{i+k+1} g_i + g_{i+k+1} f_i)."""
    M = max(len(f), len(g))
    f = list(f) + [0] * (M - len(f))
    g = list(g) + [0] * (M - len(g))
    S = []
    for k in range(M - 1):
        s = 0
        for i in range(M - k - 1):
            s += f[i + k + 1] * g[i] + g[i + k + 1] * f[i]
        S.append(s % R_MOD)
    return poly_trim(S)


def eval_pr(r, x) -> int:
    """mlpcs.rs:52-63: prod_i (r_i x^{2^i} + 1 - r_i)."""
    res, xp = 1, x % R_MOD
    for ri in r:
        res = res * (ri * xp + 1 - ri) % R_MOD
        xp = xp * xp % R_MOD
    return res


def compute_pr_ifft(r):
    """mlpcs.rs:68-78 literally: evaluate P_r on the 2^n-point subgroup, IFFT,
    trim.  O(4^n) here; use only for small n."""
    n = len(r)
    N = 1 << n
    w = two_adic_root(n)
    evals = [eval_pr(r, pow(w, k, R_MOD)) for k in range(N)]
    return poly_trim(ntt(evals, inverse=True))


def compute_pr(r):
    """O(2^n): P_r's coefficients are the eq table (identity checked against
    compute_pr_ifft and the KATs at mlpcs.rs:226-242)."""
    return poly_trim(fast_eq_eval_hypercube(len(r), r))


class MLEvalProof:
    """mlpcs.rs:32-44."""

    def __init__(self, evaluation_point, evaluation, s_comm, poly_opening,
                 poly_opening_inv, s_opening, s_opening_inv):
        self.evaluation_point = list(evaluation_point)
        self.evaluation = evaluation
        self.s_comm = s_comm
        self.poly_opening = poly_opening
        self.poly_opening_inv = poly_opening_inv
        self.s_opening = s_opening
        self.s_opening_inv = s_opening_inv

    @staticmethod
    def prove(poly, eval_point, kzg: KZG, t: Transcript, trace=None):
        """mlpcs.rs:83-124."""
        pr = compute_pr(eval_point)
        evaluation = sum(a * b for a, b in zip(poly, pr)) % R_MOD
        s_poly = compute_s_polynomial(poly, pr)
        s_comm = kzg.commit(s_poly)
        t.append_fr_vec(eval_point)
        t.append_fr(evaluation)
        t.append_g1(s_comm)
        r = t.draw_field_element()
        r_inv = fr_inv(r)
        if trace is not None:
            trace.update(pr=pr, s_poly=s_poly, r=r)
        return MLEvalProof(eval_point, evaluation, s_comm,
                           kzg.open(poly, r), kzg.open(poly, r_inv),
                           kzg.open(s_poly, r), kzg.open(s_poly, r_inv))

    def verify(self, commitment, kzg: KZG, t: Transcript) -> bool:
        """mlpcs.rs:126-161 (KZG checks via the trapdoor identity)."""
        t.append_fr_vec(self.evaluation_point)
        t.append_fr(self.evaluation)
        t.append_g1(self.s_comm)
        r = t.draw_field_element()
        r_inv = fr_inv(r)
        for C, op in ((commitment, self.poly_opening), (commitment, self.poly_opening_inv),
                      (self.s_comm, self.s_opening), (self.s_comm, self.s_opening_inv)):
            if not kzg.verify(C, op):
                return False
        pr_r = eval_pr(self.evaluation_point, r)
        pr_r_inv = eval_pr(self.evaluation_point, r_inv)
        lhs = self.poly_opening[1] * pr_r_inv + self.poly_opening_inv[1] * pr_r
        rhs = r * self.s_opening[1] + r_inv * self.s_opening_inv[1] + 2 * self.evaluation
        return (lhs - rhs) % R_MOD == 0


def mle_evaluate(evals, point) -> int:
    """DenseMultilinearExtension::evaluate (bit j of the index <-> point[j])."""
    t = [e % R_MOD for e in evals]
    for r in point:
        t = [(t[2 * i] + r * (t[2 * i + 1] - t[2 * i])) % R_MOD for i in range(len(t) // 2)]
    return t[0]


# ---------------------------------------------------------------------------
# Virtual polynomials (hyperplonk/src/utils/virtual_polynomial.rs)
# ---------------------------------------------------------------------------
class Expr:
    """VirtualPolyExpr (virtual_polynomial.rs:9-18): ('in', i) | ('const', c) |
    ('add', a, b) | ('mul', a, b).  Sub = Add(a, Mul(Const(-1), b)) (:67-77)."""

    def __init__(self, kind, *args):
        self.kind, self.args = kind, args

    @staticmethod
    def input(i):
        return Expr("in", i)

    @staticmethod
    def const(c):
        return Expr("const", c % R_MOD)

    def __add__(self, o):
        return Expr("add", self, o)

    def __mul__(self, o):
        return Expr("mul", self, o)

    def __sub__(self, o):
        return Expr("add", self, Expr("mul", Expr.const(-1), o))

    def evaluate(self, g):
        """virtual_polynomial.rs:22-37."""
        k = self.kind
        if k == "in":
            return g[self.args[0]] % R_MOD
        if k == "const":
            return self.args[0]
        a = self.args[0].evaluate(g)
        b = self.args[1].evaluate(g)
        return (a + b) % R_MOD if k == "add" else a * b % R_MOD

    def evaluate_poly(self, gp):
        """evaluate_expr_poly (virtual_polynomial.rs:300-320) on univariate polys."""
        k = self.kind
        if k == "in":
            return poly_trim(gp[self.args[0]])
        if k == "const":
            return poly_trim([self.args[0]])
        a = self.args[0].evaluate_poly(gp)
        b = self.args[1].evaluate_poly(gp)
        return poly_add(a, b) if k == "add" else poly_mul(a, b)

    def degree(self):
        k = self.kind
        if k == "in":
            return 1
        if k == "const":
            return 0
        a, b = self.args[0].degree(), self.args[1].degree()
        return max(a, b) if k == "add" else a + b


class VirtualPolynomialStore:
    """virtual_polynomial.rs:142-331 (tables as lists of canonical ints)."""

    def __init__(self, num_vars):
        self.num_vars = num_vars
        self.polynomials = []
        self.virtual_polys = []

    def allocate_polynomial(self, evals):
        assert len(evals) == 1 << self.num_vars
        self.polynomials.append([e % R_MOD for e in evals])
        return len(self.polynomials) - 1

    def new_virtual_from_input(self, g):
        self.virtual_polys.append(Expr.input(g))
        return len(self.virtual_polys) - 1

    def new_virtual_from_virtual(self, v):
        self.virtual_polys.append(self.virtual_polys[v])
        return len(self.virtual_polys) - 1

    def new_virtual_from_expr(self, e):
        self.virtual_polys.append(e)
        return len(self.virtual_polys) - 1

    def add_in_place(self, f, g):
        self.virtual_polys[f] = self.virtual_polys[f] + Expr.input(g)

    def add_const_in_place(self, f, c):
        self.virtual_polys[f] = self.virtual_polys[f] + Expr.const(c)

    def sub_in_place(self, f, g):
        self.virtual_polys[f] = self.virtual_polys[f] + (Expr.const(-1) * Expr.input(g))

    def mul_in_place(self, f, g):
        self.virtual_polys[f] = self.virtual_polys[f] * Expr.input(g)

    def mul_const_in_place(self, f, c):
        self.virtual_polys[f] = self.virtual_polys[f] * Expr.const(c)

    def evaluate_point(self, g_evals, h):
        return self.virtual_polys[h].evaluate(g_evals)


# ---------------------------------------------------------------------------
# Sumcheck / zero-check (hyperplonk/src/piops/{sumcheck,zerocheck}.rs)
# ---------------------------------------------------------------------------
class SumcheckProof:
    def __init__(self, num_vars, claimed_sum, r_polys):
        self.num_vars, self.claimed_sum, self.r_polys = num_vars, claimed_sum, r_polys

    @staticmethod
    def prove(num_vars, store: VirtualPolynomialStore, h, claimed_sum, t: Transcript):
        """sumcheck.rs:28-114, reference-structured: per pair (2p, 2p+1) each table
        becomes the linear poly low + X(high-low); the round message is
        sum_p h(...) as a trimmed coefficient-form polynomial; bit 0 binds first."""
        t.append_u64(num_vars)
        t.append_fr(claimed_sum)
        expr = store.virtual_polys[h]
        gs = [list(g) for g in store.polynomials]
        r_polys, point = [], []
        final = 0
        for i in reversed(range(num_vars)):
            msg = []
            for p in range(1 << i):
                lin = [poly_trim([g[2 * p], g[2 * p + 1] - g[2 * p]]) for g in gs]
                msg = poly_add(msg, expr.evaluate_poly(lin))
            t.append_poly(msg)
            r_polys.append(msg)
            r = t.draw_field_element()
            point.append(r)
            gs = [[(g[2 * p] + r * (g[2 * p + 1] - g[2 * p])) % R_MOD
                   for p in range(1 << i)] for g in gs]
            if i == 0:
                final = expr.evaluate([g[0] for g in gs])
        return SumcheckProof(num_vars, claimed_sum, r_polys), (point, final)

    @staticmethod
    def prove_fast(num_vars, store: VirtualPolynomialStore, h, claimed_sum, t: Transcript):
        """Evaluation-form prover producing the identical proof: evaluate h at
        t = 0..d per pair, sum, interpolate exactly, trim."""
        t.append_u64(num_vars)
        t.append_fr(claimed_sum)
        expr = store.virtual_polys[h]
        d = expr.degree()
        gs = [list(g) for g in store.polynomials]
        r_polys, point = [], []
        final = 0
        for i in reversed(range(num_vars)):
            sums = [0] * (d + 1)
            for p in range(1 << i):
                lows = [g[2 * p] for g in gs]
                diffs = [g[2 * p + 1] - g[2 * p] for g in gs]
                for tt in range(d + 1):
                    sums[tt] += expr.evaluate([lo + tt * df for lo, df in zip(lows, diffs)])
            msg = interpolate_consecutive([s % R_MOD for s in sums])
            t.append_poly(msg)
            r_polys.append(msg)
            r = t.draw_field_element()
            point.append(r)
            gs = [[(g[2 * p] + r * (g[2 * p + 1] - g[2 * p])) % R_MOD
                   for p in range(1 << i)] for g in gs]
            if i == 0:
                final = expr.evaluate([g[0] for g in gs])
        return SumcheckProof(num_vars, claimed_sum, r_polys), (point, final)

    def verify(self, t: Transcript):
        """sumcheck.rs:116-150 -> (point, evaluation) or raises ValueError."""
        t.append_u64(self.num_vars)
        t.append_fr(self.claimed_sum)
        v = self.claimed_sum % R_MOD
        point = []
        for rp in self.r_polys:
            if (poly_eval(rp, 0) + poly_eval(rp, 1) - v) % R_MOD != 0:
                raise ValueError("Sumcheck polynomial does not sum to previous value")
            t.append_poly(rp)
            r = t.draw_field_element()
            point.append(r)
            v = poly_eval(rp, r)
        return point, v


def interpolate_consecutive(vals):
    """Coefficients of the unique degree-<len(vals) polynomial with p(t)=vals[t],
    t = 0..d (Lagrange, exact), trimmed."""
    n = len(vals)
    coeffs = [0] * n
    for j in range(n):
        num = [1]
        den = 1
        for m in range(n):
            if m == j:
                continue
            num = poly_mul(num, [(-m) % R_MOD, 1]) or [0]
            den = den * (j - m) % R_MOD
        scale = vals[j] * fr_inv(den) % R_MOD
        for i, c in enumerate(num):
            coeffs[i] = (coeffs[i] + c * scale) % R_MOD
    return poly_trim(coeffs)


class ZeroCheckProof:
    def __init__(self, num_vars, sumcheck_proof):
        self.num_vars, self.sumcheck_proof = num_vars, sumcheck_proof

    @staticmethod
    def prove(store: VirtualPolynomialStore, h, t: Transcript, fast=True):
        """zerocheck.rs:14-49 (mutates `store`: +eq table, +virtual poly)."""
        n = store.num_vars
        z = [t.draw_field_element() for _ in range(n)]
        eq = fast_eq_eval_hypercube(n, z)
        eq_idx = store.allocate_polynomial(eq)
        h_hat = store.new_virtual_from_virtual(h)
        store.mul_in_place(h_hat, eq_idx)
        prover = SumcheckProof.prove_fast if fast else SumcheckProof.prove
        proof, (point, ev) = prover(n, store, h_hat, 0, t)
        e = eq_eval(z, point)
        return ZeroCheckProof(n, proof), (point, ev * fr_inv(e) % R_MOD)

    def verify(self, t: Transcript):
        """zerocheck.rs:51-76."""
        z = [t.draw_field_element() for _ in range(self.num_vars)]
        if self.sumcheck_proof.claimed_sum % R_MOD != 0:
            raise ValueError("Sumcheck claimed sum is not zero")
        if self.sumcheck_proof.num_vars != self.num_vars:
            raise ValueError("num_vars mismatch")
        point, v = self.sumcheck_proof.verify(t)
        return point, v * fr_inv(eq_eval(z, point)) % R_MOD


# ---------------------------------------------------------------------------
# Logup PIOPs (hyperplonk/src/piops/{multiset_check,set_inclusion,
# permutation_check,lookup}.rs)
# ---------------------------------------------------------------------------
LOOKUP_SUBSET, LOOKUP_EQUALITY = "subset", "equality"


def logup_column(store: VirtualPolynomialStore, h, beta, m=None):
    """multiset_check.rs:43-95 / set_inclusion.rs:93-131: per row
    m(x) / (beta + h(x)) (h, m: virtual-polynomial indices; m = 1 when None).  The reference calls
    `.inverse().unwrap()`, i.e. panics on a zero denominator: ZeroDivisionError."""
    n = 1 << store.num_vars
    den = []
    for i in range(n):
        g = [p[i] for p in store.polynomials]
        d = (beta + store.evaluate_point(g, h)) % R_MOD
        if d == 0:
            raise ZeroDivisionError("logup denominator is zero (inverse().unwrap())")
        den.append(d)
    # Montgomery batch inversion (same values as n separate inversions)
    pre, acc = [], 1
    for d in den:
        acc = acc * d % R_MOD
        pre.append(acc)
    inv = fr_inv(acc)
    out = [0] * n
    for i in reversed(range(n)):
        out[i] = inv * (pre[i - 1] if i else 1) % R_MOD
        inv = inv * den[i] % R_MOD
    if m is not None:
        for i in range(n):
            g = [p[i] for p in store.polynomials]
            out[i] = out[i] * store.evaluate_point(g, m) % R_MOD
    return out


class MultisetEqualityProof:
    """multiset_check.rs:18-24."""

    def __init__(self, cl, cr, sumcheck_proof, open_left, open_right):
        self.denom_left_commitment, self.denom_right_commitment = cl, cr
        self.sumcheck_proof = sumcheck_proof
        self.opening_proof_denom_left, self.opening_proof_denom_right = open_left, open_right

    @staticmethod
    def prove(store: VirtualPolynomialStore, h_left, h_right, t: Transcript, kzg: KZG,
              mode=LOOKUP_EQUALITY, multiplicities=None):
        """multiset_check.rs:28-181 (mutates `store`: +3 tables, +1 virtual poly)."""
        n = store.num_vars
        beta = t.draw_field_element()
        left = logup_column(store, h_left, beta)
        if mode == LOOKUP_SUBSET:
            assert multiplicities is not None, "Multiplicities polynomial must be provided"
            right = logup_column(store, h_right, beta, multiplicities)
        else:
            assert multiplicities is None, "Multiplicities polynomial must not be provided"
            right = logup_column(store, h_right, beta)
        cl, cr = kzg.commit(left), kzg.commit(right)
        t.append_g1(cl)
        t.append_g1(cr)
        lam = t.draw_field_element()
        alpha = t.draw_field_element()
        dl = store.allocate_polynomial(left)
        dr = store.allocate_polynomial(right)
        m = store.virtual_polys[multiplicities] if mode == LOOKUP_SUBSET else Expr.const(1)
        zc = (Expr.input(dl) * (Expr.const(beta) + store.virtual_polys[h_left]) - Expr.const(1)
              + Expr.const(lam) * (Expr.input(dr) * (Expr.const(beta)
                                                     + store.virtual_polys[h_right]) - m))
        z = [t.draw_field_element() for _ in range(n)]
        eq_idx = store.allocate_polynomial(fast_eq_eval_hypercube(n, z))
        h_hat = store.new_virtual_from_expr(zc)
        store.mul_in_place(h_hat, eq_idx)
        store.mul_const_in_place(h_hat, alpha)
        store.add_in_place(h_hat, dl)
        store.sub_in_place(h_hat, dr)
        sc, (point, _ev) = SumcheckProof.prove_fast(n, store, h_hat, 0, t)
        ol = MLEvalProof.prove(left, point, kzg, t)
        orr = MLEvalProof.prove(right, point, kzg, t)
        return MultisetEqualityProof(cl, cr, sc, ol, orr), point

    def verify(self, t: Transcript, kzg: KZG, left_claim, right_claim,
               mode=LOOKUP_EQUALITY, mult_claim=None):
        """multiset_check.rs:183-283.  Claims are (point, evaluation); raises
        ValueError with the reference's message on rejection."""
        beta = t.draw_field_element()
        t.append_g1(self.denom_left_commitment)
        t.append_g1(self.denom_right_commitment)
        lam = t.draw_field_element()
        alpha = t.draw_field_element()
        z = [t.draw_field_element() for _ in range(len(left_claim[0]))]
        if self.sumcheck_proof.claimed_sum % R_MOD != 0:
            raise ValueError("Multiset equality sumcheck claimed sum is not zero")
        point, ev = self.sumcheck_proof.verify(t)
        okl = self.opening_proof_denom_left.verify(self.denom_left_commitment, kzg, t)
        okr = self.opening_proof_denom_right.verify(self.denom_right_commitment, kzg, t)
        if not okl or not okr:
            raise ValueError("Multiset equality opening proof verification failed")
        if (self.opening_proof_denom_left.evaluation_point != point
                or self.opening_proof_denom_right.evaluation_point != point):
            raise ValueError("Multiset equality opening proof evaluation point does not match")
        if list(left_claim[0]) != point or list(right_claim[0]) != point:
            raise ValueError("Multiset equality h evaluation point does not match sumcheck")
        m = 1
        if mode == LOOKUP_SUBSET:
            if mult_claim is None:
                raise AssertionError("Multiplicities evaluation must be provided in subset mode")
            if list(mult_claim[0]) != point:
                raise ValueError("Multiset equality multiplicities evaluation point mismatch")
            m = mult_claim[1]
        dl = self.opening_proof_denom_left.evaluation
        dr = self.opening_proof_denom_right.evaluation
        zc = dl * (beta + left_claim[1]) - 1 + lam * (dr * (beta + right_claim[1]) - m)
        final = (zc * eq_eval(z, left_claim[0]) * alpha + dl - dr) % R_MOD
        if final != ev % R_MOD:
            raise ValueError("Multiset equality final evaluation does not match sumcheck")


class SetInclusionProof:
    """set_inclusion.rs:52-61."""

    def __init__(self, cl, cr, scl, scr, ol, orr):
        self.denom_left_commitment, self.denom_right_commitment = cl, cr
        self.sumcheck_proof_left, self.sumcheck_proof_right = scl, scr
        self.opening_proof_denom_left, self.opening_proof_denom_right = ol, orr

    @staticmethod
    def prove(store_left: VirtualPolynomialStore, h_left, store_right: VirtualPolynomialStore,
              h_right, multiplicities, t: Transcript, kzg: KZG):
        """set_inclusion.rs:74-235 -> (proof, (left point, right point))."""
        nl, nr = store_left.num_vars, store_right.num_vars
        gamma = t.draw_field_element()  # logup_eval_point
        left = logup_column(store_left, h_left, gamma)
        right = logup_column(store_right, h_right, gamma, multiplicities)
        cl, cr = kzg.commit(left), kzg.commit(right)
        t.append_g1(cl)
        t.append_g1(cr)
        z1 = [t.draw_field_element() for _ in range(nl)]
        alpha = t.draw_field_element()
        dl = store_left.allocate_polynomial(left)
        dr = store_right.allocate_polynomial(right)
        m_expr = store_right.virtual_polys[multiplicities]
        hl = store_left.virtual_polys[h_left]
        hr = store_right.virtual_polys[h_right]
        eq1 = store_left.allocate_polynomial(fast_eq_eval_hypercube(nl, z1))
        el = (Expr.input(dl) * (Expr.const(gamma) + hl) - Expr.const(1))
        el = el * Expr.input(eq1) + Expr.input(dl) * Expr.const(alpha)
        vl = store_left.new_virtual_from_expr(el)
        sum_l = sum(left) % R_MOD * alpha % R_MOD
        scl, (pl, _) = SumcheckProof.prove_fast(nl, store_left, vl, sum_l, t)
        z2 = [t.draw_field_element() for _ in range(nr)]
        beta = t.draw_field_element()
        eq2 = store_right.allocate_polynomial(fast_eq_eval_hypercube(nr, z2))
        er = Expr.input(dr) * (Expr.const(gamma) + hr) - m_expr
        er = er * Expr.input(eq2) + Expr.input(dr) * Expr.const(beta)
        vr = store_right.new_virtual_from_expr(er)
        sum_r = sum(right) % R_MOD * beta % R_MOD
        scr, (pr, _) = SumcheckProof.prove_fast(nr, store_right, vr, sum_r, t)
        ol = MLEvalProof.prove(left, pl, kzg, t)
        orr = MLEvalProof.prove(right, pr, kzg, t)
        return SetInclusionProof(cl, cr, scl, scr, ol, orr), (pl, pr)

    def verify(self, t: Transcript, kzg: KZG, h_left_claim, h_right_claim, mult_claim):
        """set_inclusion.rs:237-349 (claims are (point, evaluation))."""
        nl, nr = len(h_left_claim[0]), len(h_right_claim[0])
        gamma = t.draw_field_element()
        t.append_g1(self.denom_left_commitment)
        t.append_g1(self.denom_right_commitment)
        z1 = [t.draw_field_element() for _ in range(nl)]
        alpha = t.draw_field_element()
        pl, evl = self.sumcheck_proof_left.verify(t)
        z2 = [t.draw_field_element() for _ in range(nr)]
        beta = t.draw_field_element()
        pr, evr = self.sumcheck_proof_right.verify(t)
        if not self.opening_proof_denom_left.verify(self.denom_left_commitment, kzg, t):
            raise ValueError("Left denominator opening proof failed")
        if not self.opening_proof_denom_right.verify(self.denom_right_commitment, kzg, t):
            raise ValueError("Right denominator opening proof failed")
        dl = self.opening_proof_denom_left.evaluation
        dr = self.opening_proof_denom_right.evaluation
        if pl != self.opening_proof_denom_left.evaluation_point:
            raise ValueError("Left sumcheck point does not match PCS opening point")
        if (list(h_left_claim[0]) != pl or list(h_right_claim[0]) != pr
                or list(mult_claim[0]) != pr):
            raise ValueError("Mismatched evaluation points for set inclusion")
        if pr != self.opening_proof_denom_right.evaluation_point:
            raise ValueError("Right sumcheck point does not match PCS opening point")
        lz = dl * (gamma + h_left_claim[1]) - 1
        if (lz * eq_eval(pl, z1) + alpha * dl - evl) % R_MOD != 0:
            raise ValueError("Left sumcheck evaluation mismatch")
        rz = dr * (gamma + h_right_claim[1]) - mult_claim[1]
        if (rz * eq_eval(pr, z2) + beta * dr - evr) % R_MOD != 0:
            raise ValueError("Right sumcheck evaluation mismatch")
        v1 = self.sumcheck_proof_left.claimed_sum * fr_inv(alpha) % R_MOD
        v2 = self.sumcheck_proof_right.claimed_sum * fr_inv(beta) % R_MOD
        if v1 != v2:
            raise ValueError("Log-derivative sums do not match")


def permutation_check_prove(store, h_left, h_right, id_indices, perm_indices, t, kzg):
    """permutation_check.rs:13-59 -> (MultisetEqualityProof, point)."""
    n = store.num_vars
    assert len(id_indices) == 1 << n and len(perm_indices) == 1 << n
    id_ref = store.allocate_polynomial(id_indices)
    perm_ref = store.allocate_polynomial(perm_indices)
    alpha = t.draw_field_element()
    lh = store.new_virtual_from_virtual(h_left)
    store.mul_const_in_place(lh, alpha)
    store.add_in_place(lh, id_ref)
    rh = store.new_virtual_from_virtual(h_right)
    store.mul_const_in_place(rh, alpha)
    store.add_in_place(rh, perm_ref)
    return MultisetEqualityProof.prove(store, lh, rh, t, kzg, LOOKUP_EQUALITY, None)


def permutation_check_verify(proof, t, kzg, left_claim, right_claim, id_claim, perm_claim):
    """permutation_check.rs:61-93."""
    alpha = t.draw_field_element()
    lh = (left_claim[0], (id_claim[1] + alpha * left_claim[1]) % R_MOD)
    rh = (right_claim[0], (perm_claim[1] + alpha * right_claim[1]) % R_MOD)
    proof.verify(t, kzg, lh, rh, LOOKUP_EQUALITY, None)


def lookup_prove(source_store, source_cols, dest_store, dest_cols, multiplicities, t, kzg):
    """lookup.rs:28-84 -> (SetInclusionProof, (left point, right point))."""
    assert len(source_cols) == len(dest_cols)
    n = len(source_cols)
    t.append_u64(n)
    assert n > 0
    alpha = t.draw_field_element()
    ap = [pow(alpha, i, R_MOD) for i in range(n)]
    bl = source_store.virtual_polys[source_cols[0]]
    br = dest_store.virtual_polys[dest_cols[0]]
    for i in range(1, n):
        bl = bl + Expr.const(ap[i]) * source_store.virtual_polys[source_cols[i]]
        br = br + Expr.const(ap[i]) * dest_store.virtual_polys[dest_cols[i]]
    vl = source_store.new_virtual_from_expr(bl)
    vr = dest_store.new_virtual_from_expr(br)
    return SetInclusionProof.prove(source_store, vl, dest_store, vr, multiplicities, t, kzg)


def lookup_verify(proof, t, kzg, source_claims, dest_claims, mult_claim):
    """lookup.rs:87-141 (claims are (point, evaluation))."""
    n = len(source_claims)
    if len(dest_claims) != n:
        raise ValueError("Mismatched lookup evaluation vector lengths")
    t.append_u64(n)
    alpha = t.draw_field_element()
    ap = [pow(alpha, i, R_MOD) for i in range(n)]
    sp, dp = list(source_claims[0][0]), list(dest_claims[0][0])
    for c in source_claims:
        if list(c[0]) != sp:
            raise ValueError("Lookup evaluation points for columns are inconsistent")
    se = sum(c[1] * a for c, a in zip(source_claims, ap)) % R_MOD
    de = sum(c[1] * a for c, a in zip(dest_claims, ap)) % R_MOD
    proof.verify(t, kzg, (sp, se), (dp, de), mult_claim)


# ---------------------------------------------------------------------------
# Deterministic synthetic inputs: splitmix64 -> xoshiro256**
# ---------------------------------------------------------------------------
class Xoshiro256ss:
    M64 = (1 << 64) - 1

    def __init__(self, seed: int):
        s = seed & self.M64
        st = []
        for _ in range(4):
            s = (s + 0x9E3779B97F4A7C15) & self.M64
            z = s
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & self.M64
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & self.M64
            st.append(z ^ (z >> 31))
        self.s = st

    def next(self) -> int:
        M = self.M64
        s = self.s
        rotl = lambda x, k: ((x << k) | (x >> (64 - k))) & M  # noqa: E731
        result = (rotl((s[1] * 5) & M, 7) * 9) & M
        t = (s[1] << 17) & M
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = rotl(s[3], 45)
        return result

    def fr(self) -> int:
        """4 LE u64 limbs, top limb masked to 62 bits, reject if >= r."""
        while True:
            limbs = [self.next() for _ in range(4)]
            limbs[3] &= (1 << 62) - 1
            v = limbs[0] | (limbs[1] << 64) | (limbs[2] << 128) | (limbs[3] << 192)
            if v < R_MOD:
                return v


def fr_to_limbs_mont(x: int):
    """canonical Fr -> arkworks in-memory 4x u64 Montgomery limbs (LE)."""
    m = to_mont(x)
    return [(m >> (64 * i)) & ((1 << 64) - 1) for i in range(4)]
