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
