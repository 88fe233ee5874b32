"""Generate the golden fixtures in tests/golden/*.json from the oracle.

Run: python tests/golden/make_golden.py   (deterministic; seeds below)

The oracle (oracle/quill_oracle.py) is the CPU restatement of the reference
pinned by the reference's own KATs (see tests/test_oracle_kats.py).  These
fixtures freeze its outputs on the reference's test inputs and on seeded random
inputs so the GPU parity tests compare against committed data.  Field elements
are stored as canonical decimal strings; G1 points as [x, y] or null.
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import quill_oracle as o  # noqa: E402

R = o.R_MOD


def s(x):
    return str(x % R)


def pt(P):
    return None if P is None else [str(P[0]), str(P[1])]


def write(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1)


def expr_to_json(e):
    if e.kind == "in":
        return ["in", e.args[0]]
    if e.kind == "const":
        return ["const", s(e.args[0])]
    return [e.kind, expr_to_json(e.args[0]), expr_to_json(e.args[1])]


def sumcheck_case(name, n, tables, expr, domain, claimed=None):
    st = o.VirtualPolynomialStore(n)
    idx = [st.allocate_polynomial(t) for t in tables]
    h = st.new_virtual_from_expr(expr)
    if claimed is None:
        claimed = sum(expr.evaluate([t[i] for t in tables]) for i in range(1 << n)) % R
    t = o.Transcript(domain)
    proof, (point, ev) = o.SumcheckProof.prove(n, st, h, claimed, t)
    return {"name": name, "num_vars": n, "tables": [[s(x) for x in tb] for tb in tables],
            "expr": expr_to_json(expr), "domain": domain.decode(), "claimed_sum": s(claimed),
            "r_polys": [[s(c) for c in rp] for rp in proof.r_polys],
            "point": [s(x) for x in point], "evaluation": s(ev),
            "final_state": t.state.hex(), "_idx": idx}


def main():
    rnd = o.Xoshiro256ss(0x5155494C4C)
    I = o.Expr.input
    # ---- sumcheck: the reference test tables (sumcheck.rs:162-188) and random
    n = 3
    g1 = [((i >> 0) & 1) + 2 * ((i >> 1) & 1) + 3 * ((i >> 2) & 1) for i in range(8)]
    g2 = [((i >> 0) & 1) * 2 * ((i >> 1) & 1) + 3 * ((i >> 0) & 1) * ((i >> 2) & 1) for i in range(8)]
    cases = [sumcheck_case("reference_g1_g2", n, [g1, g2], I(0) * I(1), b"sumcheck_test")]
    for (nv, k, ename) in ((10, 3, "g0*g1*g2"), (6, 2, "g0*g0-g1"), (1, 2, "g0*g1"),
                           (11, 4, "g0*g1*g2+g3*5")):
        tabs = [[rnd.fr() for _ in range(1 << nv)] for _ in range(k)]
        if ename == "g0*g1*g2":
            e = I(0) * I(1) * I(2)
        elif ename == "g0*g0-g1":
            e = I(0) * I(0) - I(1)
        elif ename == "g0*g1":
            e = I(0) * I(1)
        else:
            e = I(0) * I(1) * I(2) + I(3) * o.Expr.const(5)
        cases.append(sumcheck_case(f"random_n{nv}_{ename}", nv, tabs, e, b"sumcheck_bench"))
    for c in cases:
        c.pop("_idx")
    write("sumcheck.json", cases)

    # ---- zero-check: the reference tables (zerocheck.rs:89-114)
    zc = []
    for name, g2v in (("valid", [0, 1, 4, 9, 16, 25, 36, 49]), ("not_zero", [0, 1, 4, 9, 16, 25, 36, 50])):
        st = o.VirtualPolynomialStore(3)
        a = st.allocate_polynomial(list(range(8)))
        b = st.allocate_polynomial(g2v)
        h = st.new_virtual_from_input(a)
        st.mul_in_place(h, a)
        st.sub_in_place(h, b)
        t = o.Transcript(b"zerocheck_test")
        proof, (point, ev) = o.ZeroCheckProof.prove(st, h, t, fast=False)
        zc.append({"name": name, "num_vars": 3, "tables": [[s(x) for x in range(8)], [s(x) for x in g2v]],
                   "expr": expr_to_json(o.Expr.input(0) * o.Expr.input(0) - o.Expr.input(1)),
                   "domain": "zerocheck_test",
                   "r_polys": [[s(c) for c in rp] for rp in proof.sumcheck_proof.r_polys],
                   "point": [s(x) for x in point], "evaluation": s(ev),
                   "eq_table": [s(x) for x in st.polynomials[2]],
                   "final_state": t.state.hex()})
    write("zerocheck.json", zc)

    # ---- MSM: bases [t_i] g with known t_i, edge scalars
    msm = []
    for n in (1, 2, 3, 31, 32, 256):
        ts = [rnd.fr() for _ in range(n)]
        sc = [rnd.fr() for _ in range(n)]
        if n >= 3:
            sc[0], sc[1], sc[2] = 0, 1, R - 1
        if n >= 32:
            ts[5] = ts[4]       # repeated base
            sc[7] = sc[6]       # repeated scalar
            sc[8] = 200         # small u8
            sc[9] = 1 << 200
        bases = [o.g1_mul(o.G1_GEN, t) for t in ts]
        res = o.g1_mul(o.G1_GEN, sum(a * b for a, b in zip(sc, ts)))
        if n <= 32:
            assert res == o.g1_msm_naive(bases, sc)
        msm.append({"n": n, "dlogs": [s(x) for x in ts], "bases": [pt(P) for P in bases],
                    "scalars": [s(x) for x in sc], "result": pt(res)})
    write("msm.json", msm)

    # ---- eq table / compute_pr / S polynomial / inner product
    z = [rnd.fr() for _ in range(5)]
    write("eq.json", {"point": [s(x) for x in z],
                      "table": [s(x) for x in o.fast_eq_eval_hypercube(5, z)],
                      "pr_kats": {"r000": [s(x) for x in o.compute_pr([0, 0, 0])],
                                  "r101": [s(x) for x in o.compute_pr([1, 0, 1])]}})
    spoly = []
    for (nf, ng) in ((3, 3), (3, 2), (7, 5), (64, 64), (100, 37), (1, 1), (2, 1)):
        f = [rnd.fr() for _ in range(nf)]
        g = [rnd.fr() for _ in range(ng)]
        spoly.append({"f": [s(x) for x in f], "g": [s(x) for x in g],
                      "S": [s(x) for x in o.compute_s_polynomial(f, g)],
                      "ip": s(sum(a * b for a, b in zip(f, g)))})
    write("spoly.json", spoly)

    # ---- KZG commit/open with a known tau (test_kzg: p = 2 + x + 3x^2 at 5)
    tau = rnd.fr()
    kzg = o.KZG(16, tau)
    kz = []
    for poly, x in (([2, 1, 3], 5), ([rnd.fr() for _ in range(17)], rnd.fr()), ([0, 0, 0], 7),
                    ([5], 3), ([1, 2, 0, 0], 9)):
        C = kzg.commit(poly)
        xx, y, pi = kzg.open(poly, x)
        kz.append({"poly": [s(c) for c in poly], "x": s(x), "commitment": pt(C), "y": s(y),
                   "proof": pt(pi)})
    write("kzg.json", {"tau": s(tau), "max_degree": 16, "cases": kz})

    # ---- ML-PCS openings (test_mlpcs_proof n=5, zero point, degree bound)
    mls = []
    for name, nv, npt, pmode in (("n5", 5, 5, "drawn"), ("zero_point", 3, 3, "zero"),
                                 ("zero_one", 3, 3, "zero_one"), ("degree_bound", 5, 3, "drawn"),
                                 ("n8", 8, 8, "drawn")):
        poly = [rnd.fr() for _ in range(1 << nv)]
        md = 4 * (1 << nv)
        tau = rnd.fr()
        kzg = o.KZG(md, tau)
        t = o.Transcript(b"MLPCS Test")
        Cm = kzg.commit(poly)
        t.append_g1(Cm)
        if pmode == "drawn":
            point = [t.draw_field_element() for _ in range(npt)]
        elif pmode == "zero":
            point = [0] * npt
        else:
            point = [0, 1, 0]
        state_before = t.state.hex()
        trace = {}
        proof = o.MLEvalProof.prove(poly, point, kzg, t, trace)
        expected = o.mle_evaluate(poly[:1 << npt], point)
        assert proof.evaluation == expected
        vt = o.Transcript(b"MLPCS Test")
        vt.state = bytes.fromhex(state_before)
        assert proof.verify(Cm, kzg, vt)

        def op(x):
            return {"x": s(x[0]), "y": s(x[1]), "proof": pt(x[2])}
        mls.append({"name": name, "tau": s(tau), "max_degree": md, "poly": [s(x) for x in poly],
                    "commitment": pt(Cm), "point": [s(x) for x in point],
                    "state_before": state_before, "evaluation": s(proof.evaluation),
                    "s_poly": [s(x) for x in trace["s_poly"]], "r": s(trace["r"]),
                    "s_comm": pt(proof.s_comm), "poly_opening": op(proof.poly_opening),
                    "poly_opening_inv": op(proof.poly_opening_inv),
                    "s_opening": op(proof.s_opening), "s_opening_inv": op(proof.s_opening_inv),
                    "state_after": t.state.hex()})
    write("mlpcs.json", mls)
    hyperplonk_fixture()
    print("golden fixtures written to", HERE)


def hyperplonk_fixture():
    """HyperPlonk multitrace proof (test_basic_proof.rs:165-196: fibonacci +
    modified fibonacci at 8 rows) with a fixed trapdoor; the oracle verifier
    must accept it."""
    import hyperplonk_oracle as ho
    tau = 0x48595045524C4F4E4B  # tests/test_gpu_hyperplonk.py TAU
    c1, w1 = ho.fibonacci_circuit_and_trace(8)
    c2, w2 = ho.modified_fibonacci_circuit_and_trace(8)
    pcs = o.KZG(max(c1.num_cols() * c1.num_rows(), c2.num_cols() * c2.num_rows()), tau)
    hp = ho.HyperPlonk.preprocess([c1, c2], pcs)
    proof, t = hp.prove(pcs, [w1, w2])
    assert ho.hyperplonk_verify(proof, hp.to_vk(), pcs).state == t.state
    write("hyperplonk.json", {
        "rows": 8, "circuits": ["fib", "mod"], "tau": s(tau),
        "witness": [[[s(x) for x in col] for col in w] for w in (w1, w2)],
        "witness_commitments": [pt(C) for C in proof.witness_commitment],
        "id_commitments": [pt(vk.id_commitment) for vk in hp.trace_vks],
        "permutation_commitments": [pt(vk.permutation_commitment) for vk in hp.trace_vks],
        "zerocheck_r_polys": [[[s(x) for x in m] for m in tp.zero_check_proof.sumcheck_proof.r_polys]
                              for tp in proof.trace_proofs],
        "permcheck_r_polys": [[[s(x) for x in m]
                               for m in tp.permutation_check_proof.sumcheck_proof.r_polys]
                              for tp in proof.trace_proofs],
        "final_state": t.state.hex()})


if __name__ == "__main__":
    main()
