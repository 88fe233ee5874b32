"""Oracle restatement of the Logup PIOPs (multiset_check.rs, set_inclusion.rs,
permutation_check.rs, lookup.rs) checked the way the reference's own tests
check them: honest proofs verify, tampered witnesses are rejected
(multiset_check.rs:310-460, permutation_check.rs:106-333, lookup.rs:197-396,
set_inclusion.rs tests).  The reference has no golden bytes for these proofs,
so transcript bytes are "parity unpinned" beyond the KAT-pinned pieces they
are built from.  CPU only."""
import random

import pytest

import quill_oracle as o

R = o.R_MOD
TAU = 0x1234567890ABCDEF1122334455667788


def _mle(evals, point):
    return o.mle_evaluate(evals, point)


def test_logup_column_values_and_zero_denominator():
    rnd = random.Random(1)
    st = o.VirtualPolynomialStore(3)
    a = st.allocate_polynomial([rnd.randrange(R) for _ in range(8)])
    b = st.allocate_polynomial([rnd.randrange(R) for _ in range(8)])
    h = st.new_virtual_from_expr(o.Expr.input(a) * o.Expr.input(b) + o.Expr.const(7))
    m = st.new_virtual_from_input(b)
    beta = rnd.randrange(R)
    col = o.logup_column(st, h, beta)
    colm = o.logup_column(st, h, beta, m)
    for i in range(8):
        d = (beta + st.polynomials[a][i] * st.polynomials[b][i] + 7) % R
        assert col[i] * d % R == 1
        assert colm[i] * d % R == st.polynomials[b][i]
    # beta + h(x) == 0 at one row: the reference's inverse().unwrap() panics
    st.polynomials[a][5] = (-(beta + 7)) * pow(st.polynomials[b][5], -1, R) % R
    with pytest.raises(ZeroDivisionError):
        o.logup_column(st, h, beta)


@pytest.mark.parametrize("tamper", [False, True])
def test_multiset_equality_roundtrip(tamper):
    """multiset_check.rs:310-460 at num_vars = 4."""
    rnd = random.Random(7)
    n = 4
    kzg = o.KZG(1 << n, TAU)
    left = [rnd.randrange(R) for _ in range(1 << n)]
    right = list(left)
    rnd.shuffle(right)
    if tamper:
        right[0] = (right[0] + 1) % R
    st = o.VirtualPolynomialStore(n)
    li, ri = st.allocate_polynomial(left), st.allocate_polynomial(right)
    hl, hr = st.new_virtual_from_input(li), st.new_virtual_from_input(ri)
    t = o.Transcript(b"multiset_equality_test")
    proof, point = o.MultisetEqualityProof.prove(st, hl, hr, t, kzg)
    assert len(st.polynomials) == 5 and len(st.virtual_polys) == 3  # store mutation
    tv = o.Transcript(b"multiset_equality_test")
    lc, rc = (point, _mle(left, point)), (point, _mle(right, point))
    if tamper:
        with pytest.raises(ValueError):
            proof.verify(tv, kzg, lc, rc)
    else:
        proof.verify(tv, kzg, lc, rc)
        assert tv.state == t.state


def test_multiset_subset_mode_roundtrip():
    """LookupMode::Subset with a multiplicities polynomial."""
    rnd = random.Random(9)
    n = 3
    kzg = o.KZG(1 << n, TAU)
    table = [rnd.randrange(R) for _ in range(1 << n)]
    mult = [0] * (1 << n)
    src = []
    for _ in range(1 << n):
        j = rnd.randrange(1 << n)
        src.append(table[j])
        mult[j] += 1
    st = o.VirtualPolynomialStore(n)
    si, ti, mi = (st.allocate_polynomial(v) for v in (src, table, mult))
    hl, hr, hm = (st.new_virtual_from_input(i) for i in (si, ti, mi))
    t = o.Transcript(b"subset")
    proof, pt = o.MultisetEqualityProof.prove(st, hl, hr, t, kzg, o.LOOKUP_SUBSET, hm)
    tv = o.Transcript(b"subset")
    proof.verify(tv, kzg, (pt, _mle(src, pt)), (pt, _mle(table, pt)), o.LOOKUP_SUBSET,
                 (pt, _mle(mult, pt)))


@pytest.mark.parametrize("tamper", [False, True])
def test_permutation_check_roundtrip(tamper):
    """permutation_check.rs:106-333: copy constraints between two columns."""
    rnd = random.Random(3)
    n = 3
    N = 1 << n
    kzg = o.KZG(2 * N, TAU)
    perm = list(range(N))
    rnd.shuffle(perm)
    left = [rnd.randrange(R) for _ in range(N)]
    right = [left[perm[i]] for i in range(N)]
    if tamper:
        right[1] = (right[1] + 5) % R
    ids, perms = list(range(N)), [perm[i] for i in range(N)]
    st = o.VirtualPolynomialStore(n)
    li, ri = st.allocate_polynomial(left), st.allocate_polynomial(right)
    hl, hr = st.new_virtual_from_input(li), st.new_virtual_from_input(ri)
    t = o.Transcript(b"perm")
    proof, pt = o.permutation_check_prove(st, hl, hr, ids, perms, t, kzg)
    tv = o.Transcript(b"perm")
    args = (tv, kzg, (pt, _mle(left, pt)), (pt, _mle(right, pt)), (pt, _mle(ids, pt)),
            (pt, _mle(perms, pt)))
    if tamper:
        with pytest.raises(ValueError):
            o.permutation_check_verify(proof, *args)
    else:
        o.permutation_check_verify(proof, *args)


@pytest.mark.parametrize("tamper", [False, True])
def test_lookup_byte_xor_roundtrip(tamper):
    """lookup.rs:197-396 (byte XOR 42 table, 2 columns), scaled to 2^5 source rows."""
    rnd = random.Random(42)
    ns, nd = 5, 8
    kzg = o.KZG(1 << nd, TAU)
    c1, c2 = list(range(256)), [i ^ 42 for i in range(256)]
    bytes_ = [rnd.randrange(256) for _ in range(1 << ns)]
    s1, s2 = list(bytes_), [b ^ 42 for b in bytes_]
    mult = [0] * 256
    for b in bytes_:
        mult[b] += 1
    if tamper:
        s2[3] = (s2[3] + 1) % R
    ss, ds = o.VirtualPolynomialStore(ns), o.VirtualPolynomialStore(nd)
    a1, a2 = ss.allocate_polynomial(s1), ss.allocate_polynomial(s2)
    d1, d2, dm = ds.allocate_polynomial(c1), ds.allocate_polynomial(c2), ds.allocate_polynomial(mult)
    sc = [ss.new_virtual_from_input(a1), ss.new_virtual_from_input(a2)]
    dc = [ds.new_virtual_from_input(d1), ds.new_virtual_from_input(d2)]
    m = ds.new_virtual_from_input(dm)
    t = o.Transcript(b"lookup")
    proof, (pl, pr) = o.lookup_prove(ss, sc, ds, dc, m, t, kzg)
    tv = o.Transcript(b"lookup")
    args = (tv, kzg, [(pl, _mle(s1, pl)), (pl, _mle(s2, pl))],
            [(pr, _mle(c1, pr)), (pr, _mle(c2, pr))], (pr, _mle(mult, pr)))
    if tamper:
        with pytest.raises(ValueError):
            o.lookup_verify(proof, *args)
    else:
        o.lookup_verify(proof, *args)


def test_c_logup_column_matches_python_oracle():
    """The C restatement (per-row binary-Euclid inverse, bench.py's CPU
    baseline) agrees with the Python restatement, and panics on zero."""
    import numpy as np
    import oracle_c
    rnd = random.Random(11)
    n = 64
    cols = [[rnd.randrange(R) for _ in range(n)] for _ in range(3)]
    a, beta = rnd.randrange(R), rnd.randrange(R)
    mont = lambda xs: np.array([o.fr_to_limbs_mont(x) for x in xs], dtype=np.uint64)  # noqa: E731
    out, _ = oracle_c.logup_column_arrays(mont(cols[0]), mont(cols[1]), mont(cols[2]),
                                          o.fr_to_limbs_mont(a), o.fr_to_limbs_mont(beta))
    st = o.VirtualPolynomialStore(6)
    for c in cols:
        st.allocate_polynomial(c)
    h = st.new_virtual_from_expr(o.Expr.input(0) + o.Expr.const(a) * o.Expr.input(1))
    m = st.new_virtual_from_input(2)
    ref = o.logup_column(st, h, beta, m)
    got = [o.from_mont(sum(int(v) << (64 * i) for i, v in enumerate(row))) for row in out]
    assert got == ref
    cols[0][9] = (-(beta + a * cols[1][9])) % R
    with pytest.raises(ZeroDivisionError):
        oracle_c.logup_column_arrays(mont(cols[0]), mont(cols[1]), mont(cols[2]),
                                     o.fr_to_limbs_mont(a), o.fr_to_limbs_mont(beta))
