"""Parity of the gfx950 path (through the C-ABI) with the oracle and the
committed golden fixtures.  Bit-exact: field elements, affine G1 points,
round messages and transcript states must be identical."""
import json
import os
import random

import pytest

import quill_oracle as o

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
R = o.R_MOD


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def P(j):
    return None if j is None else (int(j[0]), int(j[1]))


def ints(xs):
    return [int(x) for x in xs]


def build_mirror_expr(j):
    from quill_amd import VirtualPolyExpr as E
    if j[0] == "in":
        return E.Input(j[1])
    if j[0] == "const":
        return E.Const(int(j[1]))
    a, b = build_mirror_expr(j[1]), build_mirror_expr(j[2])
    return a + b if j[0] == "add" else a * b


def build_oracle_expr(j):
    if j[0] == "in":
        return o.Expr.input(j[1])
    if j[0] == "const":
        return o.Expr.const(int(j[1]))
    return o.Expr(j[0], build_oracle_expr(j[1]), build_oracle_expr(j[2]))


# ---------------------------------------------------------------- SRS / MSM
def test_srs_generate_matches_oracle(dev):
    from quill_amd import Srs
    tau = 0x1234567890ABCDEF
    srs = Srs.generate(dev, tau, 40)
    pts = srs.download()
    for i, Q in enumerate(pts):
        assert Q == o.g1_mul(o.G1_GEN, pow(tau, i, R)), i


@pytest.mark.parametrize("case", range(6))
def test_msm_golden(dev, case):
    from quill_amd import Srs
    c = load("msm.json")[case]
    srs = Srs.upload(dev, [P(b) for b in c["bases"]])
    assert srs.msm(ints(c["scalars"])) == P(c["result"])


def test_msm_edge_scalars(dev):
    from quill_amd import Srs
    rnd = random.Random(3)
    ts = [rnd.randrange(R) for _ in range(300)]
    bases = [o.g1_mul(o.G1_GEN, t) for t in ts]
    bases[10] = None  # infinity base
    ts[10] = 0
    srs = Srs.upload(dev, bases)

    def expect(sc):
        return o.g1_mul(o.G1_GEN, sum(a * b for a, b in zip(sc, ts)))
    for sc in ([0] * 300, [1] * 300, [R - 1] * 300, [7] * 300, [rnd.randrange(256) for _ in range(300)],
               [rnd.randrange(R) for _ in range(300)], [1 << 253] * 300):
        assert srs.msm(sc) == expect(sc)
    # msm_unchecked truncates to the shorter input (kzg.rs:72)
    sc = [rnd.randrange(R) for _ in range(100)]
    assert srs.msm(sc) == expect(sc)
    assert srs.msm([]) is None


@pytest.mark.parametrize("n", [1, 2, 33, 1000, 4097, 1 << 16])
def test_kzg_commit_trapdoor(dev, n):
    """commit(p) == [p(tau)] g for an SRS built from a known tau."""
    from quill_amd import KZG
    rnd = random.Random(n)
    tau = rnd.randrange(R)
    kzg = KZG.trusted_setup(n - 1, tau, dev)
    poly = [rnd.randrange(R) for _ in range(n)]
    C = kzg.commit(poly)
    assert C == o.g1_mul(o.G1_GEN, o.poly_eval(poly, tau))
    # prefix commit (shorter polynomial, bases truncated)
    assert kzg.commit(poly[: n // 2]) == o.g1_mul(o.G1_GEN, o.poly_eval(poly[: n // 2], tau))


@pytest.mark.parametrize("pieces", [2, 3, 7])
def test_host_commit_in_pieces(dev, pieces, monkeypatch):
    """qg_kzg_commit / qg_msm_g1 from host memory with the upload split into
    pieces overlapped with the pieces' accumulation (QG_MSM_PIECES; 4 by
    default from 2^22 scalars): same point as the single-piece path, ragged
    last piece and msm_unchecked truncation included."""
    from quill_amd import KZG, Srs
    rnd = random.Random(pieces)
    tau = rnd.randrange(R)
    n = 1000
    kzg = KZG.trusted_setup(n - 1, tau, dev)
    poly = [rnd.randrange(R) for _ in range(n)]
    want = o.g1_mul(o.G1_GEN, o.poly_eval(poly, tau))
    monkeypatch.setenv("QG_MSM_PIECES", str(pieces))
    assert kzg.commit(poly) == want
    assert kzg.commit(poly[:333]) == o.g1_mul(o.G1_GEN, o.poly_eval(poly[:333], tau))
    srs = Srs.upload(dev, [o.g1_mul(o.G1_GEN, pow(tau, i, R)) for i in range(50)])
    sc = [rnd.randrange(R) for _ in range(80)]  # longer than the bases: truncated
    assert srs.msm(sc) == o.g1_mul(o.G1_GEN, o.poly_eval(sc[:50], tau))


def test_kzg_commit_rejects_oversize(dev):
    from quill_amd import KZG, QuillGpuError
    kzg = KZG.trusted_setup(4, 5, dev)
    with pytest.raises(QuillGpuError):
        kzg.commit([1] * 6)  # kzg.rs:62-65 panics


def test_msm_large_trapdoor(dev):
    """2^20 MSM (config C2 size) against [<s, tau^i>] g; SRS from tau."""
    from quill_amd import DeviceVec, Srs
    n = 1 << 20
    tau = 987654321987654321
    srs = Srs.generate(dev, tau, n)
    v = DeviceVec(dev, n).fill_random(42)
    got = srs.msm_dev(v)
    sc = v.to_list()
    acc = 0
    tp = 1
    for s_ in sc:
        acc = (acc + s_ * tp) % R
        tp = tp * tau % R
    assert got == o.g1_mul(o.G1_GEN, acc)


# ---------------------------------------------------------------- PCS building blocks
def test_eq_table_golden(dev):
    g = load("eq.json")
    assert dev.eq_table(ints(g["point"])) == ints(g["table"])
    assert dev.eq_table([1, 0, 1]) == [0, 0, 0, 0, 0, 1, 0, 0]
    rnd = random.Random(4)
    z = [rnd.randrange(R) for _ in range(14)]
    tab = dev.eq_table(z)
    for i in (0, 1, 777, (1 << 14) - 1):
        assert tab[i] == o.eq_eval([(i >> j) & 1 for j in range(14)], z)


def test_s_polynomial_and_inner_product_golden(dev):
    for c in load("spoly.json"):
        f, g = ints(c["f"]), ints(c["g"])
        S = o.poly_trim(dev.s_polynomial(f, g))
        assert S == ints(c["S"])
        assert dev.inner_product(f, g) == int(c["ip"])


def test_s_polynomial_large(dev):
    rnd = random.Random(12)
    f = [rnd.randrange(R) for _ in range(3000)]
    g = [rnd.randrange(R) for _ in range(2048)]
    S = dev.s_polynomial(f, g)
    assert len(S) == 2999
    # spot-check coefficients of the correlation form
    for k in (0, 1, 1000, 2047, 2998):
        exp = sum((f[i + k + 1] * (g[i] if i < len(g) else 0) +
                   (g[i + k + 1] if i + k + 1 < len(g) else 0) * f[i])
                  for i in range(3000 - k - 1)) % R
        assert S[k] == exp


@pytest.mark.parametrize("nf,ng", [(512, 300), (1000, 999), (1 << 15, 1 << 15),
                                   ((1 << 15) + 3, (1 << 14) - 5), (5000, 1),
                                   ((1 << 18) + 3, (1 << 17) + 9)])
def test_s_polynomial_multi_pass(dev, nf, ng):
    """The NTT pass plan (mlpcs.hip ntt_plan) runs 10 stages in the first LDS
    pass (1024-element tiles) and up to 7 in each later one: M = 512 is one
    pass (2^10 points), M = 1000 two (10 + 1, the 1-stage pass on 512-wide
    runs), 2^16 / 2^17-point transforms two (10 + 6, 10 + 7), M = 2^18 + 3
    (a 2^20-point transform) three (10 + 7 + 3) like every 2^20+ ML-open.  Spot
    coefficients of S_k = sum_i (f_{i+k+1} g_i + g_{i+k+1} f_i)
    (ipa.rs:122-157)."""
    rnd = random.Random(nf + ng)
    f = [rnd.randrange(R) for _ in range(nf)]
    g = [rnd.randrange(R) for _ in range(ng)]
    M = max(nf, ng)
    fp = f + [0] * (M - nf)
    gp = g + [0] * (M - ng)
    S = dev.s_polynomial(f, g)
    assert len(S) == M - 1
    for k in sorted({k for k in (0, 1, 2, 777, M // 2, M - 3, M - 2) if k < M - 1}):
        exp = sum(fp[i + k + 1] * gp[i] + gp[i + k + 1] * fp[i] for i in range(M - k - 1)) % R
        assert S[k] == exp, k


def test_kzg_open_golden(dev):
    from quill_amd import KZG
    g = load("kzg.json")
    kzg = KZG.trusted_setup(g["max_degree"], int(g["tau"]), dev)
    for c in g["cases"]:
        poly = ints(c["poly"])
        assert kzg.commit(poly) == P(c["commitment"])
        op = kzg.open_univariate(poly, int(c["x"]))
        assert op.x == int(c["x"]) and op.y == int(c["y"]) and op.proof == P(c["proof"])


def test_kzg_open_large(dev):
    from quill_amd import KZG
    rnd = random.Random(8)
    n = 20000
    tau = rnd.randrange(R)
    kzg = KZG.trusted_setup(n, tau, dev)
    poly = [rnd.randrange(R) for _ in range(n)]
    x = rnd.randrange(R)
    op = kzg.open_univariate(poly, x)
    y = o.poly_eval(poly, x)
    assert op.y == y
    # proof = [q(tau)] g with q(tau) = (p(tau) - y) / (tau - x)
    q_tau = (o.poly_eval(poly, tau) - y) * o.fr_inv(tau - x) % R
    assert op.proof == o.g1_mul(o.G1_GEN, q_tau)


@pytest.mark.parametrize("case", range(5))
def test_mle_open_golden(dev, case):
    from quill_amd import KZG, Transcript
    c = load("mlpcs.json")[case]
    kzg = KZG.trusted_setup(c["max_degree"], int(c["tau"]), dev)
    poly = ints(c["poly"])
    assert kzg.commit(poly) == P(c["commitment"])
    t = Transcript(b"MLPCS Test")
    t.state = bytes.fromhex(c["state_before"])
    proof = kzg.open(poly, ints(c["point"]), t)
    assert proof.evaluation == int(c["evaluation"])
    assert proof.s_comm == P(c["s_comm"])
    for k in ("poly_opening", "poly_opening_inv", "s_opening", "s_opening_inv"):
        op = getattr(proof, k)
        assert (op.x, op.y, op.proof) == (int(c[k]["x"]), int(c[k]["y"]), P(c[k]["proof"])), k
    assert t.state.hex() == c["state_after"]


def test_mle_open_verifies_with_oracle(dev):
    """Opening at 2^12 evals: the oracle verifier (trapdoor KZG checks) accepts."""
    from quill_amd import KZG, Transcript
    rnd = random.Random(21)
    nv = 12
    poly = [rnd.randrange(R) for _ in range(1 << nv)]
    tau = rnd.randrange(R)
    kzg = KZG.trusted_setup(1 << nv, tau, dev)
    C = kzg.commit(poly)
    t = Transcript(b"MLPCS Test")
    t.append_g1(C)
    point = [t.draw_field_element() for _ in range(nv)]
    s0 = t.state
    proof = kzg.open(poly, point, t)
    assert proof.evaluation == o.mle_evaluate(poly, point)
    okzg = o.KZG(1 << nv, tau, points=[])
    op = o.MLEvalProof(point, proof.evaluation, proof.s_comm,
                       *[(getattr(proof, k).x, getattr(proof, k).y, getattr(proof, k).proof)
                         for k in ("poly_opening", "poly_opening_inv", "s_opening", "s_opening_inv")])
    vt = o.Transcript(b"x")
    vt.state = s0
    assert op.verify(C, okzg, vt)
    assert vt.state == t.state


@pytest.mark.parametrize("n,nv", [(2, 0), (37, 0), (1 << 10, 0), (2, 1), (33, 2), (64, 3)])
def test_mle_open_short_point_matches_oracle(dev, n, nv):
    """Opening a vector longer than 2^|point| (mlpcs.rs:91-94, prefix semantics)
    incl. the empty point: pr = [1] and S is built from the whole polynomial
    (the eq-table transform must not run for nvars = 0).  Every
    field of the proof and the transcript state equal the oracle prover's."""
    from quill_amd import KZG, Transcript
    rnd = random.Random(1000 * n + nv)
    tau = rnd.randrange(R)
    poly = [rnd.randrange(R) for _ in range(n)]
    point = [rnd.randrange(R) for _ in range(nv)]
    kzg = KZG.trusted_setup(n, tau, dev)
    # a larger open first leaves stale data in the NTT scratch buffers
    kzg.open([rnd.randrange(R) for _ in range(n)],
             [rnd.randrange(R) for _ in range(max(1, n.bit_length() - 1))], Transcript(b"stale"))
    t = Transcript(b"MLPCS short point")
    proof = kzg.open(poly, point, t)
    ot = o.Transcript(b"MLPCS short point")
    ref = o.MLEvalProof.prove(poly, point, o.KZG(n, tau, points=[]), ot)
    assert proof.evaluation == ref.evaluation
    assert proof.s_comm == ref.s_comm
    for k in ("poly_opening", "poly_opening_inv", "s_opening", "s_opening_inv"):
        op = getattr(proof, k)
        assert (op.x, op.y, op.proof) == tuple(getattr(ref, k)), k
    assert t.state == ot.state


# ---------------------------------------------------------------- sumcheck / zero-check
@pytest.mark.parametrize("case", range(5))
def test_sumcheck_golden(dev, case):
    from quill_amd import SumcheckProof, Transcript, VirtualPolynomialStore
    c = load("sumcheck.json")[case]
    st = VirtualPolynomialStore(c["num_vars"])
    for tb in c["tables"]:
        st.allocate_polynomial(ints(tb))
    h = st.new_virtual_from_expr(build_mirror_expr(c["expr"]))
    t = Transcript(c["domain"].encode())
    proof, claim = SumcheckProof.prove(c["num_vars"], st, h, int(c["claimed_sum"]), t, dev)
    assert proof.r_polys == [ints(rp) for rp in c["r_polys"]]
    assert claim.point == ints(c["point"]) and claim.evaluation == int(c["evaluation"])
    assert t.state.hex() == c["final_state"]


@pytest.mark.parametrize("case", range(2))
def test_zerocheck_golden(dev, case):
    from quill_amd import Transcript, VirtualPolynomialStore, ZeroCheckProof
    c = load("zerocheck.json")[case]
    st = VirtualPolynomialStore(3)
    for tb in c["tables"]:
        st.allocate_polynomial(ints(tb))
    h = st.new_virtual_from_expr(build_mirror_expr(c["expr"]))
    t = Transcript(b"zerocheck_test")
    proof, claim = ZeroCheckProof.prove(st, h, t, dev)
    assert proof.sumcheck_proof.r_polys == [ints(rp) for rp in c["r_polys"]]
    assert claim.point == ints(c["point"]) and claim.evaluation == int(c["evaluation"])
    assert t.state.hex() == c["final_state"]
    # store mutation mirrors zerocheck.rs:27-29
    assert st.polynomials[2] == ints(c["eq_table"]) and len(st.virtual_polys) == 2


@pytest.mark.parametrize("nv,expr", [(2, "prod3"), (5, "mixed"), (12, "prod3"), (13, "mixed"),
                                     (14, "const_only"), (9, "square_sub")])
def test_sumcheck_vs_live_oracle(dev, nv, expr):
    """Random tables crossing the tail threshold (2^12) and odd expressions."""
    from quill_amd import SumcheckProof, Transcript, VirtualPolyExpr as E, VirtualPolynomialStore
    rnd = random.Random(nv * 31 + len(expr))
    k = 4
    tabs = [[rnd.randrange(R) for _ in range(1 << nv)] for _ in range(k)]
    if expr == "prod3":
        me, oe = E.Input(0) * E.Input(1) * E.Input(2), o.Expr.input(0) * o.Expr.input(1) * o.Expr.input(2)
    elif expr == "mixed":
        me = E.Input(3) * (E.Input(0) + E.Const(7)) * E.Input(1) - E.Input(2) * E.Const(3)
        oe = o.Expr.input(3) * (o.Expr.input(0) + o.Expr.const(7)) * o.Expr.input(1) - \
            o.Expr.input(2) * o.Expr.const(3)
    elif expr == "const_only":
        me, oe = E.Const(11) * E.Const(3), o.Expr.const(11) * o.Expr.const(3)
    else:
        me, oe = E.Input(1) * E.Input(1) - E.Input(1), o.Expr.input(1) * o.Expr.input(1) - o.Expr.input(1)
    claimed = rnd.randrange(R)  # need not be the true sum: the prover is deterministic
    st = VirtualPolynomialStore(nv)
    ost = o.VirtualPolynomialStore(nv)
    for tb in tabs:
        st.allocate_polynomial(tb)
        ost.allocate_polynomial(tb)
    h = st.new_virtual_from_expr(me)
    oh = ost.new_virtual_from_expr(oe)
    t, ot = Transcript(b"sumcheck_bench"), o.Transcript(b"sumcheck_bench")
    proof, claim = SumcheckProof.prove(nv, st, h, claimed, t, dev)
    if nv <= 9:
        oproof, (opt, oev) = o.SumcheckProof.prove_fast(nv, ost, oh, claimed, ot)
        assert proof.r_polys == oproof.r_polys
        assert (claim.point, claim.evaluation) == (opt, oev)
        assert t.state == ot.state
    else:
        # size-independent properties: the oracle verifier replays the transcript
        true_sum = None
        vt = o.Transcript(b"sumcheck_bench")
        prf = o.SumcheckProof(nv, claimed, proof.r_polys)
        # the first round must sum to the claimed value only if the claim is true;
        # recompute the true sum and re-prove with it for the verifier check
        true_sum = sum(oe.evaluate([tb[i] for tb in tabs]) for i in range(1 << nv)) % R
        st2 = VirtualPolynomialStore(nv)
        for tb in tabs:
            st2.allocate_polynomial(tb)
        h2 = st2.new_virtual_from_expr(me)
        t2 = Transcript(b"sumcheck_bench")
        proof2, claim2 = SumcheckProof.prove(nv, st2, h2, true_sum, t2, dev)
        prf = o.SumcheckProof(nv, true_sum, proof2.r_polys)
        vpt, vev = prf.verify(vt)
        assert vpt == claim2.point and vev == claim2.evaluation
        assert vt.state == t2.state
        g_at = [o.mle_evaluate(tb, vpt) for tb in tabs]
        assert oe.evaluate(g_at) == vev


def test_sumcheck_2p16_property(dev):
    """2^16 vars-size tables, degree 3: verifier replay + final claim = h(MLE(point))."""
    from quill_amd import SumcheckProof, Transcript, VirtualPolyExpr as E, VirtualPolynomialStore
    from quill_amd import DeviceVec
    nv = 16
    vecs = [DeviceVec(dev, 1 << nv).fill_random(100 + i) for i in range(3)]
    tabs = [v.to_list() for v in vecs]
    true_sum = sum(a * b % R * c for a, b, c in zip(*tabs)) % R
    st = VirtualPolynomialStore(nv)
    for tb in tabs:
        st.allocate_polynomial(tb)
    h = st.new_virtual_from_expr(E.Input(0) * E.Input(1) * E.Input(2))
    t = Transcript(b"sumcheck_bench")
    proof, claim = SumcheckProof.prove(nv, st, h, true_sum, t, dev)
    vt = o.Transcript(b"sumcheck_bench")
    vpt, vev = o.SumcheckProof(nv, true_sum, proof.r_polys).verify(vt)
    assert vpt == claim.point and vev == claim.evaluation and vt.state == t.state
    g_at = [o.mle_evaluate(tb, vpt) for tb in tabs]
    assert g_at[0] * g_at[1] % R * g_at[2] % R == vev


def test_mle_open_dev_matches_host_entry(dev):
    """qg_mle_open_dev on a device vector == qg_mle_open on the same host values."""
    from quill_amd import KZG, DeviceVec, Transcript
    rnd = random.Random(33)
    nv = 10
    n = (1 << nv) - 3  # a prefix shorter than the hypercube
    kzg = KZG.trusted_setup(1 << nv, rnd.randrange(R), dev)
    vec = DeviceVec(dev, 1 << nv).fill_random(99)
    poly = vec.to_list(n)
    point = [rnd.randrange(R) for _ in range(nv)]
    t1, t2 = Transcript(b"dev"), Transcript(b"dev")
    p1 = kzg.open(poly, point, t1)
    p2 = kzg.open_dev(vec, n, point, t2)
    assert p1 == p2 and t1.state == t2.state


def test_mle_open_unchanged_reuses_transform(dev):
    """qg_mle_open_dev_ex(QG_OPEN_UNCHANGED) gives the same proofs as fresh
    openings: repeated openings of one buffer (the transform reused), an
    interleaved opening of another buffer (the kept transform is not that
    buffer's: recomputed), and a changed buffer opened without the flag."""
    from quill_amd import KZG, DeviceVec, Transcript
    rnd = random.Random(34)
    nv = 11
    kzg = KZG.trusted_setup(1 << nv, rnd.randrange(R), dev)
    a = DeviceVec(dev, 1 << nv).fill_random(7)
    b = DeviceVec(dev, 1 << nv).fill_random(8)
    pts = [[rnd.randrange(R) for _ in range(nv)] for _ in range(4)]
    seq = [(a, pts[0], False), (a, pts[1], True), (b, pts[2], False), (a, pts[3], True),
           (a, pts[0], True)]
    # the device sequence first (host-input openings in between would replace
    # the kept transform), then the reference openings from host copies
    t_fast, t_ref = Transcript(b"reuse"), Transcript(b"reuse")
    fast = [(kzg.open_dev(vec, len(vec), pt, t_fast, unchanged=u), t_fast.state)
            for vec, pt, u in seq]
    host = {id(a): a.to_list(), id(b): b.to_list()}
    for (vec, pt, _), (pf, st) in zip(seq, fast):
        assert kzg.open(host[id(vec)], pt, t_ref) == pf and t_ref.state == st
    # a changed buffer, opened without the flag, is transformed afresh
    a.fill_random(9)
    t1, t2 = Transcript(b"reuse2"), Transcript(b"reuse2")
    assert kzg.open_dev(a, len(a), pts[1], t1) == kzg.open(a.to_list(), pts[1], t2)


@pytest.mark.parametrize("n,nv,live", [(64, 6, 40), (64, 6, 0), (100, 5, 50), (64, 6, 1)])
def test_mle_open_zero_tail_matches_oracle(dev, n, nv, live):
    """Vectors whose trailing entries are zero (only the first `live` nonzero;
    live = 0: the zero polynomial): the ML opening commits S over all its
    coefficients and runs the quotients on the trimmed lengths read back after
    the commitment's synchronization (mlpcs.hip mle_open_device), and every
    field of the proof and the transcript state equal the oracle prover's
    (DensePolynomial trims, kzg.rs:75-96).  The same buffer is then opened
    again with QG_OPEN_UNCHANGED (the trimmed length remembered), and after
    its tail changes, without the flag (the length recomputed)."""
    from quill_amd import KZG, DeviceVec, Transcript
    rnd = random.Random(7000 + 10 * n + live)
    tau = rnd.randrange(R)
    kzg = KZG.trusted_setup(max(n, 1 << nv), tau, dev)
    okzg = o.KZG(max(n, 1 << nv), tau, points=[])

    def check(poly, vec, point, unchanged):
        t = Transcript(b"zero tail")
        proof = kzg.open_dev(vec, n, point, t, unchanged=unchanged)
        ot = o.Transcript(b"zero tail")
        ref = o.MLEvalProof.prove(poly, point, okzg, ot)
        assert proof.evaluation == ref.evaluation and proof.s_comm == ref.s_comm
        for k in ("poly_opening", "poly_opening_inv", "s_opening", "s_opening_inv"):
            op = getattr(proof, k)
            assert (op.x, op.y, op.proof) == tuple(getattr(ref, k)), k
        assert t.state == ot.state

    poly = [rnd.randrange(R) for _ in range(live)] + [0] * (n - live)
    vec = DeviceVec.from_list(dev, poly)
    pts = [[rnd.randrange(R) for _ in range(nv)] for _ in range(3)]
    check(poly, vec, pts[0], False)
    check(poly, vec, pts[1], True)
    poly2 = poly[:]
    poly2[n - 1] = rnd.randrange(1, R)  # the tail now ends in a nonzero entry
    vec2 = DeviceVec.from_list(dev, poly2)
    vec.copy_from(vec2)
    check(poly2, vec, pts[2], False)
    vec.close()
    vec2.close()


def test_microbench_entry_points(dev):
    """qg_microbench_fq_mul / qg_microbench_fetch (the bench's compute peak and
    the PMC probe's FETCH_SIZE calibration) run and report positive rates"""
    assert dev.microbench_fq_mul() > 1e9
    g, s = dev.microbench_fetch(1 << 16, 1 << 16)
    assert g > 0 and s > 0


def test_ctx_counter_reports_plan_refetches(dev):
    """qg_ctx_counter: the MSM plan-copy refetch count is a readable integer
    after a batched MSM (an ML opening: one S commitment + four quotient
    MSMs), unknown names read 0; the opening still verifies."""
    from quill_amd import KZG, Transcript
    rnd = random.Random(31)
    poly = [rnd.randrange(R) for _ in range(1 << 10)]
    tau = rnd.randrange(R)
    kzg = KZG.trusted_setup(1 << 10, tau, dev)
    point = [rnd.randrange(R) for _ in range(10)]
    proof = kzg.open(poly, point, Transcript(b"counter"))
    assert proof.evaluation == o.mle_evaluate(poly, point)
    assert dev.counter("msm_plan_refetch") >= 0
    assert dev.counter("no_such_counter") == 0


def test_s_polynomial_size_cycle_keeps_twiddles_fresh(dev):
    """Transforms of alternating sizes on one context: every regrowth of the
    twiddle scratch frees a table whose address a later table (forward or
    inverse, same logn) may get again, so the per-address pyramid and
    bit-reversed caches must be rebuilt with the table (mlpcs.hip
    ntt_twiddles), not served by address (an inverse NTT on forward
    twiddles failed the 2^14-row HyperPlonk opening check).  Spot coefficients
    against the correlation formula after every size change."""
    rnd = random.Random(99)
    for nf in (40000, 70000, 40000, 140000, 40000, 70000, 1 << 15):
        f = [rnd.randrange(R) for _ in range(nf)]
        g = [rnd.randrange(R) for _ in range(nf // 2)]
        gp = g + [0] * (nf - len(g))
        S = dev.s_polynomial(f, g)
        for k in (0, nf // 3, nf - 2):
            exp = sum(f[i + k + 1] * gp[i] + gp[i + k + 1] * f[i] for i in range(nf - k - 1)) % R
            assert S[k] == exp, (nf, k)


@pytest.mark.parametrize("seed", [0, 1])
def test_mle_open_batch_matches_sequential_and_oracle(dev, seed):
    """qg_mle_open_batch_dev: K openings with the S and quotient commitments
    as two MSM batches and the transcript steps in item order.  Items of
    different lengths and variable counts (n < 2^nv, n = 2^nv, n > 2^nv),
    zero-tailed and zero vectors, one vector opened twice (the second with
    QG_OPEN_UNCHANGED, as HyperPlonk opens its witness per column).  Every
    proof and the final transcript state equal K successive open_dev calls,
    and the oracle prover's (mlpcs.rs:83-124) on the same transcript."""
    from quill_amd import KZG, DeviceVec, Transcript
    rnd = random.Random(9100 + seed)
    tau = rnd.randrange(R)
    kzg = KZG.trusted_setup(1 << 9, tau, dev)
    okzg = o.KZG(1 << 9, tau, points=[])
    shapes = [(256, 8, 256), (200, 8, 120), (64, 6, 0), (300, 8, 300), (512, 9, 511), (32, 6, 32)]
    polys, vecs, items = [], [], []
    for n, nv, live in shapes:
        p = [rnd.randrange(R) for _ in range(live)] + [0] * (n - live)
        polys.append(p)
        vecs.append(DeviceVec.from_list(dev, p))
        items.append((len(polys) - 1, nv, False))
    items.append((0, 8, True))  # vector 0 again, unchanged
    pts = [[rnd.randrange(R) for _ in range(nv)] for _, nv, _ in items]
    batch_in = [(vecs[i], len(polys[i]), pt, u) for (i, _, u), pt in zip(items, pts)]
    tb = Transcript(b"open batch")
    got = kzg.open_batch_dev(batch_in, tb)
    ts = Transcript(b"open batch")
    seq = [kzg.open_dev(v, n, pt, ts, unchanged=u) for v, n, pt, u in batch_in]
    assert got == seq
    assert tb.state == ts.state
    ot = o.Transcript(b"open batch")
    for (i, _, _), pt, proof in zip(items, pts, got):
        ref = o.MLEvalProof.prove(polys[i], pt, okzg, ot)
        assert proof.evaluation == ref.evaluation and proof.s_comm == ref.s_comm
        for k in ("poly_opening", "poly_opening_inv", "s_opening", "s_opening_inv"):
            op = getattr(proof, k)
            assert (op.x, op.y, op.proof) == tuple(getattr(ref, k)), k
    assert tb.state == ot.state
    # a second batch on the same context: its first item reuses the length the
    # first batch left remembered (vector 0, unchanged), its last one must not
    # (vector 1 was opened in between), as with successive single openings
    batch2 = [(vecs[0], len(polys[0]), pts[0], True), (vecs[1], len(polys[1]), pts[1], False),
              (vecs[0], len(polys[0]), [rnd.randrange(R) for _ in range(8)], True)]
    got2 = kzg.open_batch_dev(batch2, tb)
    ts2 = Transcript(b"open batch 2")
    tb2 = Transcript(b"open batch 2")
    got2b = kzg.open_batch_dev(batch2, tb2)
    seq2 = [kzg.open_dev(v, n, pt, ts2, unchanged=u) for v, n, pt, u in batch2]
    assert got2b == seq2 and tb2.state == ts2.state
    for (v, n, pt, _), proof in zip(batch2, got2):
        ref = o.MLEvalProof.prove(polys[vecs.index(v)], pt, okzg, ot)
        assert proof.evaluation == ref.evaluation
        for k in ("poly_opening", "poly_opening_inv", "s_opening", "s_opening_inv"):
            op = getattr(proof, k)
            assert (op.x, op.y, op.proof) == tuple(getattr(ref, k)), k
    assert tb.state == ot.state
    for v in vecs:
        v.close()
