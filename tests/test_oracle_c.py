"""The oracle's C restatement (CPU baseline) agrees with the Python oracle.
CPU only."""
import random

import pytest

import quill_oracle as o

oc = pytest.importorskip("oracle_c")


@pytest.fixture(scope="module", autouse=True)
def _lib():
    try:
        oc.lib()
    except FileNotFoundError:
        pytest.skip("oracle/_build/liboracle_c.so not built (make -C oracle)")


@pytest.mark.parametrize("n", [1, 2, 3, 31, 32, 33, 200])
def test_c_msm_matches_python(n):
    rnd = random.Random(n)
    ts = [rnd.randrange(o.R_MOD) for _ in range(n)]
    bases = [o.g1_mul(o.G1_GEN, t) for t in ts]
    sc = [rnd.randrange(o.R_MOD) for _ in range(n)]
    if n > 3:
        sc[0], sc[1] = 0, o.R_MOD - 1
        bases[2], ts[2] = None, 0
        bases[3] = bases[4]
        ts[3] = ts[4]
    assert oc.msm(bases, sc) == o.g1_mul(o.G1_GEN, sum(a * b for a, b in zip(sc, ts)))


def test_c_sumcheck_matches_python():
    rnd = random.Random(2)
    nv = 6
    tabs = [[rnd.randrange(o.R_MOD) for _ in range(1 << nv)] for _ in range(3)]
    st = o.VirtualPolynomialStore(nv)
    for t in tabs:
        st.allocate_polynomial(t)
    h = st.new_virtual_from_expr(o.Expr.input(0) * o.Expr.input(1) * o.Expr.input(2))
    t = o.Transcript(b"sumcheck_bench")
    proof, (pt, ev) = o.SumcheckProof.prove_fast(nv, st, h, 77, t)
    rp, cpt, cev, cst = oc.sumcheck_prod(nv, tabs, 77, o.Transcript(b"sumcheck_bench").state)
    assert rp == proof.r_polys and cpt == pt and cev == ev and cst == t.state


def test_c_baseline_runs_small():
    r = oc.bench_msm_baseline(8)
    assert r["value"] > 0 and r["cores"] == 1 and r["kind"] == "port"


def _to_limbs(xs):
    import numpy as np
    return np.array([oc._mont(x, o.R_MOD) for x in xs], dtype=np.uint64)


def test_c_checkers_match_python():
    """The full-size checkers (Horner / MLE / sum of products / scalar mul) used
    by the headline-size GPU tests and bench.py agree with the Python oracle."""
    rnd = random.Random(5)
    nv = 7
    tabs = [[rnd.randrange(o.R_MOD) for _ in range(1 << nv)] for _ in range(3)]
    x = rnd.randrange(o.R_MOD)
    assert oc.fr_horner(_to_limbs(tabs[0]), x) == o.poly_eval(tabs[0], x)
    pt = [rnd.randrange(o.R_MOD) for _ in range(nv)]
    assert oc.fr_mle_eval(_to_limbs(tabs[1]), pt) == o.mle_evaluate(tabs[1], pt)
    # a prefix of a longer table (mlpcs.rs:91-94 semantics)
    assert oc.fr_mle_eval(_to_limbs(tabs[1]), pt[:4]) == o.mle_evaluate(tabs[1][:16], pt[:4])
    assert oc.fr_sum_prod([_to_limbs(t) for t in tabs]) == \
        sum(a * b % o.R_MOD * c for a, b, c in zip(*tabs)) % o.R_MOD
    for s in (0, 1, o.R_MOD - 1, x):
        assert oc.g1_mul(o.G1_GEN, s) == o.g1_mul(o.G1_GEN, s)
    P = o.g1_mul(o.G1_GEN, 12345)
    assert oc.g1_mul(P, x) == o.g1_mul(P, x)
    assert oc.g1_mul(None, x) is None


@pytest.mark.parametrize("nv,k", [(1, 2), (5, 3), (9, 3), (7, 4)])
def test_c_sumcheck_variants_agree(nv, k):
    """The reference-structured (DensePolynomial + FFT products) and the
    all-cores evaluation-form baselines produce the evaluation-form proof
    bit-for-bit (same transcript bytes)."""
    rnd = random.Random(nv * 10 + k)
    tabs = [[rnd.randrange(o.R_MOD) for _ in range(1 << nv)] for _ in range(k)]
    claim = rnd.randrange(o.R_MOD)
    base = oc.sumcheck_prod(nv, tabs, claim, b"\x07" * 32)
    assert oc.sumcheck_prod(nv, tabs, claim, b"\x07" * 32, variant="ref") == base
    assert oc.sumcheck_prod(nv, tabs, claim, b"\x07" * 32, variant="mt", nthreads=3) == base


def test_c_msm_mt_matches_single_thread():
    """ark-ec's parallel window split gives the single-thread MSM's point."""
    import numpy as np
    rnd = random.Random(5)
    n = 300
    ts = [rnd.randrange(o.R_MOD) for _ in range(n)]
    bases = [o.g1_mul(o.G1_GEN, t) for t in ts]
    sc = [rnd.randrange(o.R_MOD) for _ in range(n)]
    xy = np.array([oc._mont(b[0], o.P_MOD) + oc._mont(b[1], o.P_MOD) for b in bases],
                  dtype=np.uint64)
    inf = np.zeros(n, dtype=np.uint8)
    s = np.array([oc._mont(x, o.R_MOD) for x in sc], dtype=np.uint64)
    _, _, single = oc.bench_msm_arrays(xy, inf, s)
    _, multi = oc.bench_msm_arrays_mt(xy, inf, s, 4)
    assert single == multi


@pytest.mark.parametrize("nv", [0, 1, 3, 6])
def test_c_mle_open_matches_oracle(nv):
    """oc_mle_open_ref (the C restatement of MLEvalProof::prove used as the
    ML-open CPU baseline) gives the Python oracle's proof and transcript state"""
    import random
    rnd = random.Random(nv)
    R = o.R_MOD
    poly = [rnd.randrange(R) for _ in range(1 << nv)]
    pt = [rnd.randrange(R) for _ in range(nv)]
    tau = 0x5155494C4C2D53525321
    t = o.Transcript(b"mle_c")
    st0 = bytes(t.state)
    pr = o.MLEvalProof.prove(poly, pt, o.KZG(max(2, 1 << nv), tau), t)
    out, st, _ = oc.mle_open_ref(nv, poly, pt, tau, st0)
    assert out["evaluation"] == pr.evaluation and out["s_comm"] == pr.s_comm
    assert st == bytes(t.state)
    ops = (pr.poly_opening, pr.poly_opening_inv, pr.s_opening, pr.s_opening_inv)
    assert out["y"] == [op[1] for op in ops]
    assert out["proof"] == [op[2] for op in ops]


@pytest.mark.parametrize("rows", [8, 32])
def test_c_hyperplonk_matches_oracle(rows):
    """hyperplonk_c.c_backend (the C5 CPU baseline: commitments, openings,
    sumchecks, Logup columns and eq tables in C) proves exactly what the pure
    Python restatement proves: same commitments, messages, openings, final state"""
    import hyperplonk_c as hc
    import hyperplonk_oracle as ho
    tau = 0x48595045524C4F4E4B
    cws = [ho.fibonacci_circuit_and_trace(rows), ho.modified_fibonacci_circuit_and_trace(rows)]
    pcs = o.KZG(max(c.num_cols() * c.num_rows() for c, _ in cws), tau)
    hp = ho.HyperPlonk.preprocess([c for c, _ in cws], pcs)
    p1, t1 = hp.prove(pcs, [w for _, w in cws])
    with hc.c_backend(tau, pcs.max_degree + 1):
        p2, t2 = hp.prove(pcs, [w for _, w in cws])
    assert t1.state == t2.state
    assert p1.witness_commitment == p2.witness_commitment
    for a, b in zip(p1.trace_proofs, p2.trace_proofs):
        assert a.zero_check_proof.sumcheck_proof.r_polys == b.zero_check_proof.sumcheck_proof.r_polys
        ma, mb = a.permutation_check_proof, b.permutation_check_proof
        assert (ma.denom_left_commitment, ma.denom_right_commitment) == \
            (mb.denom_left_commitment, mb.denom_right_commitment)
        for x, y in zip(a.openings_zero_check + [a.opening_id, a.opening_permutation_trace],
                        b.openings_zero_check + [b.opening_id, b.opening_permutation_trace]):
            assert (x.evaluation, x.s_comm, x.poly_opening, x.s_opening_inv) == \
                (y.evaluation, y.s_comm, y.poly_opening, y.s_opening_inv)
    # the backend is restored
    assert o.KZG.commit is not hc._commit


def test_c_sumcheck_mont_entry_matches_list_entry():
    """sumcheck_prod_mont (numpy Montgomery limbs in, the 2^20 GPU parity
    test's checker) = sumcheck_prod (Python ints in)"""
    rnd = random.Random(31)
    nv = 7
    tabs = [[rnd.randrange(o.R_MOD) for _ in range(1 << nv)] for _ in range(3)]
    st = o.Transcript(b"mont-entry").state
    a = oc.sumcheck_prod(nv, tabs, 1234, st)
    for variant in ("mt", "eval"):
        b = oc.sumcheck_prod_mont(nv, [_to_limbs(t) for t in tabs], 1234, st, variant=variant)
        assert a == b
