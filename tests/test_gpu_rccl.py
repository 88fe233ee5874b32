"""The RCCL transport on a 1-GPU box (VERDICT r3 "next" 2).

RCCL refuses two ranks on one device ("Duplicate GPU detected"), so a real
multi-rank communicator needs the driver's 8-GPU node.  QG_FORCE_RCCL=1 makes a
world-1 context attach a real one-rank RCCL communicator (ncclCommInitRank with
its own unique id) and take the SHARDED code paths, whose exchanges then run
ncclAllGather and grouped ncclSend/ncclRecv instead of the single-GPU memcpy.
Every result must equal the unsharded single-context result bit for bit
(MSM: kzg.rs:72; sumcheck: sumcheck.rs:28-114; ML open with the S polynomial
split by frequency residue: mlpcs.rs:83-124 / ipa.rs:122-157)."""
import os
import random

import pytest

import quill_oracle as o

pytestmark = pytest.mark.gpu
R = o.R_MOD


@pytest.fixture(scope="module")
def rdev():
    import quill_amd as q
    old = os.environ.get("QG_FORCE_RCCL")
    os.environ["QG_FORCE_RCCL"] = "1"
    try:
        d = q.Device(0)
        d.attach_comm(0, 1, q.Device.comm_unique_id())
    finally:
        if old is None:
            os.environ.pop("QG_FORCE_RCCL")
        else:
            os.environ["QG_FORCE_RCCL"] = old
    yield d
    d.close()


def test_forced_comm_is_rccl(rdev, dev):
    assert rdev.comm_info() == {"kind": "rccl", "rank": 0, "world": 1, "sharded": True}
    assert dev.comm_info() == {"kind": "none", "rank": 0, "world": 1, "sharded": False}
    # the library really mapped librccl
    with open("/proc/self/maps") as f:
        assert "librccl" in f.read()


def test_rccl_collectives_host(rdev):
    data = bytes(range(256)) * 3
    assert rdev.allgather_bytes(data) == [data]
    assert rdev.alltoall_bytes([data]) == [data]


@pytest.mark.parametrize("logn", [11, 16])
def test_rccl_msm_matches_single(rdev, dev, logn):
    import quill_amd as q
    rnd = random.Random(logn)
    n = 1 << logn
    tau = rnd.randrange(R)
    out = []
    for d in (dev, rdev):
        srs = q.Srs.generate(d, tau, n)
        v = q.DeviceVec(d, n).fill_random(77 + logn)
        out.append(srs.msm_dev(v))
        v.close()
        srs.close()
    assert out[0] == out[1]
    assert out[0] is not None


@pytest.mark.parametrize("nv,ntab", [(9, 3), (18, 3), (20, 3), (17, 6)])
def test_rccl_sumcheck_matches_single(rdev, dev, nv, ntab):
    """run_rounds_dist at world 1: per-round ncclAllGather of the round sums,
    the gather of the folded tables, then the slice tail (or k_sc_tail)."""
    import quill_amd as q
    from quill_amd.hyperplonk import VirtualPolyExpr as E, sumcheck_prove_device
    expr = E.Input(0) * E.Input(1) * E.Input(2)
    if ntab > 3:
        expr = expr + E.Input(3) * E.Input(4) - E.Input(5) * E.Const(7)
    res = []
    for d in (dev, rdev):
        tabs = [q.DeviceVec(d, 1 << nv).fill_random(9000 + 13 * i + nv) for i in range(ntab)]
        t = q.Transcript(b"rccl-sumcheck")
        coeffs, lens, point, ev = sumcheck_prove_device(d, nv, tabs, expr, 12345, t)
        res.append((coeffs.tobytes(), lens.tobytes(), point.tobytes(), bytes(ev), t.state))
        for tb in tabs:
            tb.close()
    assert res[0] == res[1]


def test_rccl_zerocheck_matches_single(rdev, dev):
    import quill_amd as q
    from quill_amd.hyperplonk import VirtualPolyExpr as E, sumcheck_prove_tables
    rnd = random.Random(3)
    nv = 12
    g0 = [rnd.randrange(R) for _ in range(1 << nv)]
    g1 = [x * x % R for x in g0]
    me = E.Input(0) * E.Input(0) - E.Input(1)
    res = []
    for d in (dev, rdev):
        t = q.Transcript(b"rccl-zc")
        res.append((sumcheck_prove_tables(d, nv, [g0, g1], me, 0, t, zerocheck=True), t.state))
    assert res[0] == res[1]


@pytest.mark.parametrize("nv,tail_zeros", [(9, 0), (9, 131), (16, 0)])
def test_rccl_mle_open_matches_single(rdev, dev, nv, tail_zeros):
    """mle_open_sharded at world 1: the residue-split S polynomial (one block,
    half of it zero padding) and its ncclSend/ncclRecv all-to-all, the sharded
    quotients and MSMs; equal to the single-context proof and transcript."""
    import quill_amd as q
    from quill_amd import KZG, Transcript
    rnd = random.Random(nv * 10 + tail_zeros)
    N = 1 << nv
    tau = rnd.randrange(R)
    poly = [rnd.randrange(R) for _ in range(N)]
    for i in range(tail_zeros):
        poly[N - 1 - i] = 0
    point = [rnd.randrange(R) for _ in range(nv)]
    res = []
    for d in (dev, rdev):
        kzg = KZG(d, q.Srs.generate(d, tau, N), N - 1)
        vec = q.DeviceVec.from_list(d, poly)
        t = Transcript(b"rccl-open")
        res.append((kzg.open_dev(vec, N, point, t), t.state))
        vec.close()
        kzg.srs.close()
    assert res[0] == res[1]


def test_rccl_logup_matches_single(rdev, dev):
    import quill_amd as q
    from quill_amd import VirtualPolyExpr as E
    from quill_amd.logup import logup_column_device
    nv = 14
    res = []
    for d in (dev, rdev):
        tabs = [q.DeviceVec(d, 1 << nv).fill_random(555 + i) for i in range(3)]
        out = q.DeviceVec(d, 1 << nv)
        s = logup_column_device(d, nv, tabs, E.Input(0) + E.Const(5) * E.Input(1), 0xBEEF, out,
                                E.Input(2))
        res.append((s, out.to_list()))
        for tb in tabs + [out]:
            tb.close()
    assert res[0] == res[1]


def test_rccl_msm_dev_batch_matches_single(rdev, dev):
    """msm_finish_ranks_batch at world 1: one ncclAllGather of a batch's k
    partials (round 6); equal to the single-context batch"""
    import quill_amd as q
    tau = 0x5CA1AB1E
    ns = [1 << 14, 1000, 0, (1 << 13) + 5]
    out = []
    for d in (dev, rdev):
        srs = q.Srs.generate(d, tau, 1 << 14)
        vs = [q.DeviceVec(d, 1 << 14).fill_random(31 + i) for i in range(len(ns))]
        out.append(srs.msm_dev_batch(vs, ns))
        for v in vs:
            v.close()
        srs.close()
    assert out[0] == out[1]


def test_rccl_mle_open_batch_matches_single(rdev, dev):
    """mle_open_batch_sharded at world 1 (round 6: four exchanges per batch over
    ncclAllGather / grouped send-recv): the proofs and transcript state of the
    single-context batch, items of one local length incl. a zero tail"""
    import quill_amd as q
    from quill_amd import KZG, Transcript
    rnd = random.Random(66)
    nv = 12
    N = 1 << nv
    tau = rnd.randrange(R)
    polys = [[rnd.randrange(R) for _ in range(N)] for _ in range(3)]
    polys[1] = polys[1][:N - 700] + [0] * 700
    items = [(0, [rnd.randrange(R) for _ in range(nv)]), (1, [rnd.randrange(R) for _ in range(nv)]),
             (2, [rnd.randrange(R) for _ in range(nv)]), (0, [rnd.randrange(R) for _ in range(nv)])]
    res = []
    for d in (dev, rdev):
        kzg = KZG.trusted_setup(N, tau, d)
        vs = [q.DeviceVec.from_list(d, p) for p in polys]
        t = Transcript(b"rccl-open-batch")
        res.append((kzg.open_batch_dev([(vs[i], N, pt, False) for i, pt in items], t), t.state))
        for v in vs:
            v.close()
        kzg.close()
    assert res[0] == res[1]


def test_rccl_hyperplonk_matches_oracle(rdev):
    """HyperPlonk::prove (proof.rs:239-301) on the forced one-rank RCCL context:
    the sharded prover end to end (full-witness exchange, sharded commitments
    and commitment batches, zero-checks, Logup, batched sharded openings) over
    the real RCCL transport; the proof equals the oracle prover's field by
    field with the same transcript state"""
    import quill_amd as q
    from quill_amd import examples as ex
    from test_gpu_hyperplonk import TAU, _oracle_setup, assert_same_proof
    rows, which = 64, ("fib", "mod")
    opcs, ohp, ows = _oracle_setup(rows, which)
    oproof, ot = ohp.prove(opcs, ows)
    b = {"fib": ex.fibonacci_circuit_and_trace, "mod": ex.modified_fibonacci_circuit_and_trace}
    cws = [b[w](rows) for w in which]
    maxdeg = max(c.num_cols() * c.num_rows() for c, _ in cws)
    pcs = q.KZG.trusted_setup(maxdeg, TAU, rdev)
    hp = q.HyperPlonk.preprocess([c for c, _ in cws], pcs)
    proof = hp.prove(pcs, [w for _, w in cws])
    pcs.close()
    assert_same_proof(proof, oproof)
    assert hp.last_transcript.state == ot.state
