"""Expressions outside the compiled fast paths: more than 8
tables, degree above 15, monomial expansions beyond the 256-term sumcheck
image / 128-term Logup image — all taken by the generic postfix interpreter
(sumcheck.hip k_gen_eval / k_gen_table).  Bit-exact against the oracle's
reference-structured prover (sumcheck.rs:28-114, zerocheck.rs:14-49,
multiset_check.rs:43-95) and, end to end, a 16-column TransitionCircuit
(transition_circuit.rs) proved by HyperPlonk (proof.rs:239-301)."""
import random

import pytest

import hyperplonk_oracle as ho
import quill_oracle as o

pytestmark = pytest.mark.gpu
R = o.R_MOD
TAU = 0x48595045524C4F4E4B


def _pow(x, k):
    y = x
    for _ in range(k - 1):
        y = y * x
    return y


def _exprs(kind):
    """(mirror expression, oracle expression, number of tables)"""
    from quill_amd import VirtualPolyExpr as E
    O = o.Expr
    if kind == "tables12":  # 12 tables, degree 3
        me = oe = None
        for i in range(12):
            c = 3 * i + 1
            a = E.Const(c) * E.Input(i) * E.Input((i + 5) % 12)
            b = O.const(c) * O.input(i) * O.input((i + 5) % 12)
            me, oe = (a, b) if me is None else (me + a, oe + b)
        me = me + E.Input(11) * E.Input(10) * E.Input(3)
        oe = oe + O.input(11) * O.input(10) * O.input(3)
        return me, oe, 12
    if kind == "deg17":  # degree 17 over 3 tables
        me = _pow(E.Input(0) * E.Input(1), 8) * E.Input(2) + E.Const(5)
        oe = _pow(O.input(0) * O.input(1), 8) * O.input(2) + O.const(5)
        return me, oe, 3
    if kind == "blowup":  # (a0 + .. + a6)^5: 462 monomials
        ms, os_ = E.Input(0), O.input(0)
        for i in range(1, 7):
            ms, os_ = ms + E.Input(i), os_ + O.input(i)
        return _pow(ms, 5) - E.Input(3), _pow(os_, 5) - O.input(3), 7
    if kind == "deg31":  # syntactic degree 31: 32 evaluation points per round
        me = _pow(E.Input(0) - E.Const(2), 31)
        oe = _pow(O.input(0) - O.const(2), 31)
        return me, oe, 1
    raise ValueError(kind)


def _stores(nv, tabs):
    from quill_amd import VirtualPolynomialStore
    st, ost = VirtualPolynomialStore(nv), o.VirtualPolynomialStore(nv)
    for tb in tabs:
        st.allocate_polynomial(tb)
        ost.allocate_polynomial(tb)
    return st, ost


@pytest.mark.parametrize("nv,kind", [(1, "tables12"), (5, "tables12"), (8, "deg17"),
                                     (7, "blowup"), (4, "deg31"), (2, "blowup")])
def test_sumcheck_generic_vs_oracle(dev, nv, kind):
    from quill_amd import SumcheckProof, Transcript
    rnd = random.Random(nv * 131 + len(kind))
    me, oe, k = _exprs(kind)
    tabs = [[rnd.randrange(R) for _ in range(1 << nv)] for _ in range(k)]
    st, ost = _stores(nv, tabs)
    h, oh = st.new_virtual_from_expr(me), ost.new_virtual_from_expr(oe)
    claimed = rnd.randrange(R)
    t, ot = Transcript(b"generic"), o.Transcript(b"generic")
    proof, claim = SumcheckProof.prove(nv, st, h, claimed, t, dev)
    oproof, (opt, oev) = o.SumcheckProof.prove(nv, ost, oh, claimed, ot)
    assert proof.r_polys == oproof.r_polys
    assert (claim.point, claim.evaluation) == (opt, oev)
    assert t.state == ot.state


@pytest.mark.parametrize("nv,kind", [(14, "tables12"), (12, "blowup")])
def test_sumcheck_generic_large_property(dev, nv, kind):
    """oracle verifier replay of a true claim + final claim = h(MLE_i(point))"""
    from quill_amd import SumcheckProof, Transcript
    from quill_amd import DeviceVec
    me, oe, k = _exprs(kind)
    vecs = [DeviceVec(dev, 1 << nv).fill_random(300 + i) for i in range(k)]
    tabs = [v.to_list() for v in vecs]
    true_sum = sum(oe.evaluate([tb[i] for tb in tabs]) for i in range(1 << nv)) % R
    st, _ = _stores(nv, tabs)
    h = st.new_virtual_from_expr(me)
    t = Transcript(b"generic")
    proof, claim = SumcheckProof.prove(nv, st, h, true_sum, t, dev)
    vt = o.Transcript(b"generic")
    vpt, vev = o.SumcheckProof(nv, true_sum, proof.r_polys).verify(vt)
    assert vpt == claim.point and vev == claim.evaluation and vt.state == t.state
    assert oe.evaluate([o.mle_evaluate(tb, vpt) for tb in tabs]) == vev


def test_zerocheck_generic_vs_oracle(dev):
    """9 inputs + eq = 10 tables: the zero-check's h * eq runs interpreted"""
    from quill_amd import Transcript, VirtualPolyExpr as E, ZeroCheckProof
    nv = 6
    rnd = random.Random(77)
    tabs = [[rnd.randrange(R) for _ in range(1 << nv)] for _ in range(8)]
    # column 8 makes h vanish on the cube: h = a0 a1 + .. + a6 a7 - a8
    tabs.append([sum(tabs[2 * j][i] * tabs[2 * j + 1][i] for j in range(4)) % R
                 for i in range(1 << nv)])
    me = E.Input(0) * E.Input(1) + E.Input(2) * E.Input(3) + E.Input(4) * E.Input(5) + \
        E.Input(6) * E.Input(7) - E.Input(8)
    O = o.Expr
    oe = O.input(0) * O.input(1) + O.input(2) * O.input(3) + O.input(4) * O.input(5) + \
        O.input(6) * O.input(7) - O.input(8)
    st, ost = _stores(nv, tabs)
    h, oh = st.new_virtual_from_expr(me), ost.new_virtual_from_expr(oe)
    t, ot = Transcript(b"zc_generic"), o.Transcript(b"zc_generic")
    zp, zclaim = ZeroCheckProof.prove(st, h, t, dev)
    ozp, (opt, oev) = o.ZeroCheckProof.prove(ost, oh, ot)
    assert zp.sumcheck_proof.r_polys == ozp.sumcheck_proof.r_polys
    assert (zclaim.point, zclaim.evaluation) == (opt, oev)
    assert t.state == ot.state


@pytest.mark.parametrize("nv,with_m", [(6, False), (12, True)])
def test_logup_generic_vs_oracle(dev, nv, with_m):
    """(a0 + .. + a7)^4 has 330 monomials (> 128): materialised by k_gen_table"""
    from quill_amd import VirtualPolyExpr as E
    from quill_amd.logup import logup_column
    rnd = random.Random(nv)
    tabs = [[rnd.randrange(R) for _ in range(1 << nv)] for _ in range(8)]
    st, ost = _stores(nv, tabs)
    ms, os_ = E.Input(0), o.Expr.input(0)
    for i in range(1, 8):
        ms, os_ = ms + E.Input(i), os_ + o.Expr.input(i)
    h, oh = st.new_virtual_from_expr(_pow(ms, 4)), ost.new_virtual_from_expr(_pow(os_, 4))
    m = om = None
    if with_m:
        m = st.new_virtual_from_expr(_pow(ms, 4) + E.Input(2))
        om = ost.new_virtual_from_expr(_pow(os_, 4) + o.Expr.input(2))
    beta = rnd.randrange(R)
    col, s = logup_column(st, h, beta, m, dev)
    ocol = o.logup_column(ost, oh, beta, om)
    assert col == ocol
    assert s == sum(ocol) % R


# ---------------------------------------------------------------- 16-column circuit
def _wide_witness(rows):
    """6 state cells x_i (cols 2i / 2i+1) + 4 witness cells t_k (cols 12 + k):
    t0 = x0 x1 x2, t1 = t0 x3 + x4, t2 = x5^5, t3 = (x0+..+x5+t0+t1)^4,
    x_i' = x_{i+1} (i < 5), x5' = t2 + t3 + x0; x_i(0) = i + 1."""
    w = [[0] * rows for _ in range(16)]
    x = [i + 1 for i in range(6)]
    for r in range(rows):
        t0 = x[0] * x[1] % R * x[2] % R
        t1 = (t0 * x[3] + x[4]) % R
        t2 = pow(x[5], 5, R)
        t3 = pow((sum(x) + t0 + t1) % R, 4, R)
        nx = x[1:] + [(t2 + t3 + x[0]) % R]
        for i in range(6):
            w[2 * i][r], w[2 * i + 1][r] = x[i], nx[i]
        for k, v in enumerate((t0, t1, t2, t3)):
            w[12 + k][r] = v
        x = nx
    return w


def _wide_circuit_device(rows):
    from quill_amd import VirtualPolyExpr as E
    from quill_amd.frontend import TransitionCircuit
    c = TransitionCircuit(rows)
    xs = [c.allocate_state_cell() for _ in range(6)]
    ts = [c.allocate_witness_cell() for _ in range(4)]
    X = [s.current.to_expr() for s in xs]
    N = [s.next.to_expr() for s in xs]
    T = [t.to_expr() for t in ts]
    for i in range(6):
        c.enforce_boundary_constraint(0, X[i] - E.Const(i + 1))
    c.enforce_constraint(T[0] - X[0] * X[1] * X[2])
    c.enforce_constraint(T[1] - (T[0] * X[3] + X[4]))
    c.enforce_constraint(T[2] - _pow(X[5], 5))
    s = X[0] + X[1] + X[2] + X[3] + X[4] + X[5] + T[0] + T[1]
    c.enforce_constraint(T[3] - _pow(s, 4))
    for i in range(5):
        c.enforce_constraint(N[i] - X[i + 1])
    c.enforce_constraint(N[5] - (T[2] + T[3] + X[0]))
    assert c.num_cols() == 16
    return c


def _wide_circuit_oracle(rows):
    O = o.Expr
    c = ho.TransitionCircuit(rows)
    xs = [c.allocate_state_cell() for _ in range(6)]
    ts = [c.allocate_witness_cell() for _ in range(4)]
    X = [O.input(cur) for cur, _ in xs]
    N = [O.input(nxt) for _, nxt in xs]
    T = [O.input(t) for t in ts]
    for i in range(6):
        c.enforce_boundary_constraint(0, X[i] - O.const(i + 1))
    c.enforce_constraint(T[0] - X[0] * X[1] * X[2])
    c.enforce_constraint(T[1] - (T[0] * X[3] + X[4]))
    c.enforce_constraint(T[2] - _pow(X[5], 5))
    s = X[0] + X[1] + X[2] + X[3] + X[4] + X[5] + T[0] + T[1]
    c.enforce_constraint(T[3] - _pow(s, 4))
    for i in range(5):
        c.enforce_constraint(N[i] - X[i + 1])
    c.enforce_constraint(N[5] - (T[2] + T[3] + X[0]))
    return c


@pytest.mark.parametrize("rows", [8, 32])
def test_hyperplonk_16_column_circuit_vs_oracle(dev, rows):
    """23 tables (16 columns + 6 selectors + eq), degree 6, 330-term
    constraint: every proof field bit-exact, oracle verifier accepts"""
    from quill_amd import KZG, HyperPlonk
    from test_gpu_hyperplonk import assert_same_proof, to_oracle
    w = _wide_witness(rows)
    c = _wide_circuit_device(rows)
    oc_ = _wide_circuit_oracle(rows)
    oc_.check_constraints(w)
    pcs = KZG.trusted_setup(16 * rows, TAU, dev)
    hp = HyperPlonk.preprocess([c], pcs)
    proof = hp.prove(pcs, [w])
    opcs = o.KZG(16 * rows, TAU)
    ohp = ho.HyperPlonk.preprocess([oc_], opcs)
    oproof, ot = ohp.prove(opcs, [w])
    assert_same_proof(proof, oproof)
    assert hp.last_transcript.state == ot.state
    vt = ho.hyperplonk_verify(to_oracle(proof), ohp.to_vk(), opcs)
    assert vt.state == ot.state


def test_hyperplonk_16_column_bad_witness_raises(dev):
    """a violated 330-term constraint is found by the interpreted row check"""
    from quill_amd import KZG, HyperPlonk
    rows = 16
    w = _wide_witness(rows)
    w[15][9] = (w[15][9] + 1) % R  # t3 at row 9
    c = _wide_circuit_device(rows)
    pcs = KZG.trusted_setup(16 * rows, TAU, dev)
    hp = HyperPlonk.preprocess([c], pcs)
    with pytest.raises(ValueError, match="Recurring"):
        hp.prove(pcs, [w])
