"""Parity of the Logup path (qg_logup_column + the PIOP mirrors in
quill_amd.logup) with the oracle restatement of multiset_check.rs,
set_inclusion.rs, permutation_check.rs and lookup.rs.  Bit-exact: columns,
sums, commitments, sumcheck messages, openings and transcript states."""
import random

import pytest

import quill_oracle as o

pytestmark = pytest.mark.gpu
R = o.R_MOD
TAU = 0x1234567890ABCDEF1122334455667788


def _stores(nv, tabs, dev=None):
    """(mirror store, oracle store); dev given: the mirror's tables live in HBM"""
    from quill_amd import VirtualPolynomialStore
    st, ost = VirtualPolynomialStore(nv, dev), o.VirtualPolynomialStore(nv)
    for tb in tabs:
        st.allocate_polynomial(tb)
        ost.allocate_polynomial(tb)
    return st, ost


def _exprs(kind):
    from quill_amd import VirtualPolyExpr as E
    O = o.Expr
    if kind == "input":
        return E.Input(0), O.input(0)
    if kind == "affine":  # id + alpha * col (permutation_check.rs:34-41)
        a = 0x5EED
        return (E.Input(0) * E.Const(a) + E.Input(1),
                O.input(0) * O.const(a) + O.input(1))
    if kind == "batched":  # sum_i alpha^i col_i (lookup.rs:46-56)
        a = 0xA1FA
        return (E.Input(0) + E.Const(a) * E.Input(1) + E.Const(a * a) * E.Input(2),
                O.input(0) + O.const(a) * O.input(1) + O.const(a * a) * O.input(2))
    if kind == "product":
        return (E.Input(1) * E.Input(2) * E.Input(0) - E.Const(3),
                O.input(1) * O.input(2) * O.input(0) - O.const(3))
    if kind == "const":
        return E.Const(17), O.const(17)
    raise ValueError(kind)


@pytest.mark.parametrize("nv,kind,with_m", [
    (0, "input", False), (1, "affine", True), (3, "product", False), (6, "batched", True),
    (10, "affine", False), (11, "input", True), (12, "product", True), (13, "batched", False),
    (7, "const", False)])
def test_logup_column_vs_oracle(dev, nv, kind, with_m):
    """Ragged sizes around the 2048-row block (2^11) and every expression shape."""
    from quill_amd.logup import logup_column
    rnd = random.Random(nv * 7 + len(kind))
    tabs = [[rnd.randrange(R) for _ in range(1 << nv)] for _ in range(4)]
    st, ost = _stores(nv, tabs)
    me, oe = _exprs(kind)
    h, oh = st.new_virtual_from_expr(me), ost.new_virtual_from_expr(oe)
    m = om = None
    if with_m:
        from quill_amd import VirtualPolyExpr as E
        m = st.new_virtual_from_expr(E.Input(3) + E.Const(1))
        om = ost.new_virtual_from_expr(o.Expr.input(3) + o.Expr.const(1))
    beta = rnd.randrange(R)
    col, s = logup_column(st, h, beta, m, dev)
    ocol = o.logup_column(ost, oh, beta, om)
    assert col == ocol
    assert s == sum(ocol) % R


def test_logup_zero_denominator_is_an_error(dev):
    """inverse().unwrap() panics in the reference: the ABI returns QG_ERR_ASSERT."""
    from quill_amd import QuillGpuError, VirtualPolyExpr as E
    from quill_amd.logup import logup_column
    nv = 12
    rnd = random.Random(5)
    beta = rnd.randrange(R)
    for row in (0, 2047, 2048, 4095):
        tab = [rnd.randrange(R) for _ in range(1 << nv)]
        tab[row] = (-beta) % R
        st, _ = _stores(nv, [tab])
        h = st.new_virtual_from_expr(E.Input(0))
        with pytest.raises(QuillGpuError) as ei:
            logup_column(st, h, beta, None, dev)
        assert ei.value.code == -5


@pytest.mark.parametrize("nv", [20, 22])
def test_logup_column_large_property(dev, nv):
    """2^20 / 2^22 rows on device-resident tables: out * (beta + h) == m at rows
    sampled in the first, middle and last blocks and at random, and the returned
    sum equals the sum of the downloaded column.  At 2^22 rows (2048 blocks of
    2048) k_logup_scan runs its multi-entry segments (per > 1), which pins the
    per-segment prefix / suffix products."""
    import oracle_c as oc
    from quill_amd import DeviceVec, VirtualPolyExpr as E
    from quill_amd.field import fr_from_mont_limbs
    from quill_amd.logup import logup_column_device
    a = DeviceVec(dev, 1 << nv).fill_random(11)
    b = DeviceVec(dev, 1 << nv).fill_random(12)
    out = DeviceVec(dev, 1 << nv)
    beta = 0xBE7A
    s = logup_column_device(dev, nv, [a, b], E.Input(0) * E.Const(5) + E.Input(1), beta, out,
                            E.Input(1))
    A, B, O = a.to_numpy(), b.to_numpy(), out.to_numpy()
    assert s == oc.fr_sum_prod([O])
    n = 1 << nv
    rnd = random.Random(3)
    rows = [0, 1, 2047, 2048, 4095, n // 2 - 1, n // 2, n // 2 + 2049, n - 2049, n - 2048, n - 1]
    rows += [rnd.randrange(n) for _ in range(2000)]
    for i in rows:
        ai, bi, oi = (fr_from_mont_limbs(list(X[i])) for X in (A, B, O))
        assert oi * (beta + 5 * ai + bi) % R == bi, i
    for v in (a, b, out):
        v.close()


def _cmp_mle(gp, op):
    assert gp.evaluation_point == op.evaluation_point
    assert gp.evaluation == op.evaluation and gp.s_comm == op.s_comm
    for k in ("poly_opening", "poly_opening_inv", "s_opening", "s_opening_inv"):
        g = getattr(gp, k)
        assert (g.x, g.y, g.proof) == tuple(getattr(op, k)), k


def _cmp_sumcheck(gs, os_):
    assert gs.num_vars == os_.num_vars and gs.claimed_sum == os_.claimed_sum % R
    assert gs.r_polys == os_.r_polys


@pytest.mark.parametrize("resident", [False, True])
@pytest.mark.parametrize("mode", ["equality", "subset"])
def test_multiset_equality_proof_matches_oracle(dev, mode, resident):
    """multiset_check.rs:310-385 scaled to 2^5: identical proof, point, store and
    transcript; the oracle verifier accepts the GPU proof."""
    from quill_amd import KZG, Transcript
    from quill_amd.logup import LookupMode, MultisetEqualityProof
    rnd = random.Random(77)
    nv = 5
    N = 1 << nv
    left = [rnd.randrange(R) for _ in range(N)]
    if mode == "equality":
        right = list(left)
        rnd.shuffle(right)
        tabs = [left, right]
    else:
        right = [rnd.randrange(R) for _ in range(N)]
        mult = [0] * N
        left = []
        for _ in range(N):
            j = rnd.randrange(N)
            left.append(right[j])
            mult[j] += 1
        tabs = [left, right, mult]
    st, ost = _stores(nv, tabs, dev if resident else None)
    hl, hr = st.new_virtual_from_input(0), st.new_virtual_from_input(1)
    ohl, ohr = ost.new_virtual_from_input(0), ost.new_virtual_from_input(1)
    hm = ohm = None
    gmode, omode = LookupMode.Equality, o.LOOKUP_EQUALITY
    if mode == "subset":
        hm, ohm = st.new_virtual_from_input(2), ost.new_virtual_from_input(2)
        gmode, omode = LookupMode.Subset, o.LOOKUP_SUBSET
    kzg = KZG.trusted_setup(N, TAU, dev)
    okzg = o.KZG(N, TAU)
    t, ot = Transcript(b"multiset_equality_test"), o.Transcript(b"multiset_equality_test")
    proof, pt = MultisetEqualityProof.prove(st, hl, hr, t, kzg, gmode, hm)
    oproof, opt = o.MultisetEqualityProof.prove(ost, ohl, ohr, ot, okzg, omode, ohm)
    assert pt == opt and t.state == ot.state
    assert proof.denom_left_commitment == oproof.denom_left_commitment
    assert proof.denom_right_commitment == oproof.denom_right_commitment
    _cmp_sumcheck(proof.sumcheck_proof, oproof.sumcheck_proof)
    _cmp_mle(proof.opening_proof_denom_left, oproof.opening_proof_denom_left)
    _cmp_mle(proof.opening_proof_denom_right, oproof.opening_proof_denom_right)
    polys = [p.to_list() for p in st.polynomials] if resident else st.polynomials
    assert polys == ost.polynomials and len(st.virtual_polys) == len(ost.virtual_polys)
    vt = o.Transcript(b"multiset_equality_test")
    mc = (pt, o.mle_evaluate(tabs[2], pt)) if mode == "subset" else None
    oproof.verify(vt, okzg, (pt, o.mle_evaluate(left, pt)), (pt, o.mle_evaluate(right, pt)),
                  omode, mc)


def test_multiset_tampered_is_rejected(dev):
    """multiset_check.rs:387-460: a non-permutation yields a proof the verifier rejects."""
    from quill_amd import KZG, Transcript
    from quill_amd.logup import MultisetEqualityProof
    rnd = random.Random(78)
    nv = 4
    N = 1 << nv
    left = [rnd.randrange(R) for _ in range(N)]
    right = list(left)
    rnd.shuffle(right)
    right[0] = (right[0] + 1) % R
    st, _ = _stores(nv, [left, right])
    hl, hr = st.new_virtual_from_input(0), st.new_virtual_from_input(1)
    kzg = KZG.trusted_setup(N, TAU, dev)
    t = Transcript(b"multiset_equality_test")
    proof, pt = MultisetEqualityProof.prove(st, hl, hr, t, kzg)
    okzg = o.KZG(N, TAU)

    def opening(p):
        return o.MLEvalProof(p.evaluation_point, p.evaluation, p.s_comm,
                             *[(getattr(p, k).x, getattr(p, k).y, getattr(p, k).proof)
                               for k in ("poly_opening", "poly_opening_inv", "s_opening",
                                         "s_opening_inv")])
    op = o.MultisetEqualityProof(
        proof.denom_left_commitment, proof.denom_right_commitment,
        o.SumcheckProof(nv, proof.sumcheck_proof.claimed_sum, proof.sumcheck_proof.r_polys),
        opening(proof.opening_proof_denom_left), opening(proof.opening_proof_denom_right))
    with pytest.raises(ValueError):
        op.verify(o.Transcript(b"multiset_equality_test"), okzg, (pt, o.mle_evaluate(left, pt)),
                  (pt, o.mle_evaluate(right, pt)))


def test_permutation_check_matches_oracle(dev):
    """permutation_check.rs:106-218 scaled to 2^4."""
    from quill_amd import KZG, Transcript
    from quill_amd.logup import PermutationCheckProof
    rnd = random.Random(5)
    nv = 4
    N = 1 << nv
    perm = list(range(N))
    rnd.shuffle(perm)
    left = [rnd.randrange(R) for _ in range(N)]
    right = [left[perm[i]] for i in range(N)]
    ids = list(range(N))
    st, ost = _stores(nv, [left, right])
    hl, hr = st.new_virtual_from_input(0), st.new_virtual_from_input(1)
    ohl, ohr = ost.new_virtual_from_input(0), ost.new_virtual_from_input(1)
    kzg, okzg = KZG.trusted_setup(N, TAU, dev), o.KZG(N, TAU)
    t, ot = Transcript(b"perm"), o.Transcript(b"perm")
    proof, pt = PermutationCheckProof.prove(st, hl, hr, ids, perm, t, kzg)
    oproof, opt = o.permutation_check_prove(ost, ohl, ohr, ids, perm, ot, okzg)
    assert pt == opt and t.state == ot.state
    mp = proof.multiset_equality_proof
    assert mp.denom_left_commitment == oproof.denom_left_commitment
    _cmp_sumcheck(mp.sumcheck_proof, oproof.sumcheck_proof)
    _cmp_mle(mp.opening_proof_denom_right, oproof.opening_proof_denom_right)
    o.permutation_check_verify(oproof, o.Transcript(b"perm"), okzg, (pt, o.mle_evaluate(left, pt)),
                               (pt, o.mle_evaluate(right, pt)), (pt, o.mle_evaluate(ids, pt)),
                               (pt, o.mle_evaluate(perm, pt)))


@pytest.mark.parametrize("resident", [False, True])
def test_lookup_byte_xor_matches_oracle(dev, resident):
    """lookup.rs:197-297 (XOR-42 byte table, 2 columns) with 2^6 source rows:
    set inclusion with different table sizes on both sides; host-table and
    device-resident stores."""
    from quill_amd import KZG, Transcript, VirtualPolynomialStore
    from quill_amd.logup import LookupProof
    rnd = random.Random(42)
    ns, nd = 6, 8
    c1, c2 = list(range(256)), [i ^ 42 for i in range(256)]
    by = [rnd.randrange(256) for _ in range(1 << ns)]
    s1, s2 = list(by), [b ^ 42 for b in by]
    mult = [0] * 256
    for b in by:
        mult[b] += 1
    ss, oss = _stores(ns, [s1, s2], dev if resident else None)
    ds, ods = _stores(nd, [c1, c2, mult], dev if resident else None)
    sc = [ss.new_virtual_from_input(0), ss.new_virtual_from_input(1)]
    dc = [ds.new_virtual_from_input(0), ds.new_virtual_from_input(1)]
    m = ds.new_virtual_from_input(2)
    osc = [oss.new_virtual_from_input(0), oss.new_virtual_from_input(1)]
    odc = [ods.new_virtual_from_input(0), ods.new_virtual_from_input(1)]
    om = ods.new_virtual_from_input(2)
    kzg, okzg = KZG.trusted_setup(1 << nd, TAU, dev), o.KZG(1 << nd, TAU)
    t, ot = Transcript(b"lookup"), o.Transcript(b"lookup")
    proof, (pl, pr) = LookupProof.prove(ss, sc, ds, dc, m, t, kzg)
    oproof, (opl, opr) = o.lookup_prove(oss, osc, ods, odc, om, ot, okzg)
    assert (pl, pr) == (opl, opr) and t.state == ot.state
    sp = proof.set_inclusion_proof
    assert sp.denom_left_commitment == oproof.denom_left_commitment
    assert sp.denom_right_commitment == oproof.denom_right_commitment
    _cmp_sumcheck(sp.sumcheck_proof_left, oproof.sumcheck_proof_left)
    _cmp_sumcheck(sp.sumcheck_proof_right, oproof.sumcheck_proof_right)
    _cmp_mle(sp.opening_proof_denom_left, oproof.opening_proof_denom_left)
    _cmp_mle(sp.opening_proof_denom_right, oproof.opening_proof_denom_right)
    o.lookup_verify(oproof, o.Transcript(b"lookup"), okzg,
                    [(pl, o.mle_evaluate(s1, pl)), (pl, o.mle_evaluate(s2, pl))],
                    [(pr, o.mle_evaluate(c1, pr)), (pr, o.mle_evaluate(c2, pr))],
                    (pr, o.mle_evaluate(mult, pr)))
