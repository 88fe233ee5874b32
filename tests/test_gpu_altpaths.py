"""The alternate kernels kept beside the defaults, each checked bit
for bit against the default path on the same inputs:
  * k_sc_tail, the streaming sumcheck tail: QG_SC_OLD_TAIL=1 on one context, and
    the sharded prover whose gathered tail does not fit the slice tail (8 source
    tables at nvars >= 15 over 8 loopback ranks);
  * k_logup_fused, the one-pass Logup column (QG_LOGUP_FUSED=1);
  * the replicated S polynomial in the sharded ML opening (QG_S_REPLICATED=1).
  * an MSM batch in stream order (QG_MSM_PIPE=0) instead of on the two side
    streams.
The switches are read per call, so the tests toggle them in-process."""
import contextlib
import os
import random

import numpy as np
import pytest

import quill_oracle as o

pytestmark = pytest.mark.gpu
R = o.R_MOD


@contextlib.contextmanager
def env(name, value):
    old = os.environ.get(name)
    os.environ[name] = value
    try:
        yield
    finally:
        if old is None:
            os.environ.pop(name)
        else:
            os.environ[name] = old


def _prove(dev, nv, tabs, expr, label):
    import quill_amd as q
    from quill_amd.hyperplonk import sumcheck_prove_device
    t = q.Transcript(label)
    coeffs, lens, point, ev = sumcheck_prove_device(dev, nv, tabs, expr, 777, t)
    return coeffs.tobytes(), lens.tobytes(), point.tobytes(), bytes(ev), t.state


@pytest.mark.parametrize("nv,ntab", [(12, 3), (18, 3), (17, 8)])
def test_old_tail_matches_slice_tail(dev, nv, ntab):
    import quill_amd as q
    from quill_amd.hyperplonk import VirtualPolyExpr as E
    expr = E.Input(0) * E.Input(1) * E.Input(2)
    for i in range(3, ntab):
        expr = expr + E.Input(i) * E.Const(i)
    tabs = [q.DeviceVec(dev, 1 << nv).fill_random(31 * nv + i) for i in range(ntab)]
    a = _prove(dev, nv, tabs, expr, b"tail-ab")
    with env("QG_SC_OLD_TAIL", "1"):
        b = _prove(dev, nv, tabs, expr, b"tail-ab")
    for t in tabs:
        t.close()
    assert a == b


@pytest.mark.parametrize("world,nv", [(8, 17), (4, 16)])
def test_sharded_k8_tail_matches_single(world, nv):
    """8 source tables: the gathered 2^15-entry tail exceeds what the slice tail
    covers with 8 slots (and the loopback's 1/world CU share), so run_rounds_dist
    falls back to k_sc_tail; its proof equals the single-context proof."""
    import quill_amd as q
    from quill_amd.hyperplonk import VirtualPolyExpr as E, sumcheck_prove_tables
    from test_gpu_multirank import run_ranks
    lw = world.bit_length() - 1
    N, NL = 1 << nv, 1 << (nv - lw)
    dev0 = q.Device(0)
    tabs = [q.DeviceVec(dev0, N).fill_random(500 + i) for i in range(8)]
    host = [t.to_list() for t in tabs]
    for t in tabs:
        t.close()
    me = E.Input(0) * E.Input(1) * E.Input(2) + E.Input(3) * E.Input(4) * E.Input(5) \
        - E.Input(6) * E.Input(7)
    claimed = random.Random(nv).randrange(R)
    ref = sumcheck_prove_tables(dev0, nv, host, me, claimed, q.Transcript(b"k8"))
    dev0.close()

    def fn(d, rank, world):
        return sumcheck_prove_tables(d, nv, [tb[rank * NL:(rank + 1) * NL] for tb in host], me,
                                     claimed, q.Transcript(b"k8"))
    for got in run_ranks(world, fn):
        assert got == ref


@pytest.mark.parametrize("nv", [11, 13, 16])
def test_logup_fused_matches_default(dev, nv):
    import quill_amd as q
    from quill_amd import VirtualPolyExpr as E
    from quill_amd.logup import logup_column_device
    tabs = [q.DeviceVec(dev, 1 << nv).fill_random(88 + 5 * i + nv) for i in range(3)]
    res = []
    for fused in ("0", "1"):
        out = q.DeviceVec(dev, 1 << nv)
        with env("QG_LOGUP_FUSED", fused):
            s = logup_column_device(dev, nv, tabs, E.Input(0) + E.Const(0xA1FA) * E.Input(1),
                                    0xBE7A, out, E.Input(2))
        res.append((s, out.to_numpy().tobytes()))
        out.close()
    for t in tabs:
        t.close()
    assert res[0] == res[1]


@pytest.mark.parametrize("world", [2, 4])
def test_replicated_s_matches_split(world):
    import quill_amd as q
    from quill_amd import KZG, Transcript
    from test_gpu_multirank import run_ranks
    rnd = random.Random(900 + world)
    nv = 10
    N = 1 << nv
    L = N // world
    tau = rnd.randrange(R)
    poly = [rnd.randrange(R) for _ in range(N)]
    point = [rnd.randrange(R) for _ in range(nv)]

    def fn(d, rank, world):
        kzg = KZG(d, q.Srs.generate(d, tau, L, offset=rank * L), N - 1)
        vec = q.DeviceVec.from_list(d, poly[rank * L:(rank + 1) * L])
        t = Transcript(b"srep")
        pr = kzg.open_dev(vec, L, point, t)
        vec.close()
        kzg.srs.close()
        return pr, t.state
    split = run_ranks(world, fn)
    with env("QG_S_REPLICATED", "1"):
        rep = run_ranks(world, fn)
    assert split == rep
    assert all(x == split[0] for x in split)


@pytest.mark.parametrize("n,small", [((1 << 11) + 3, False), (5000, False), (5000, True),
                                     (1, False), (7, True), ((1 << 16) + 1, False)])
@pytest.mark.parametrize("mode", ["QG_MSM_PF", "QG_MSM_COOP"])
def test_alternate_accumulate_matches_default(n, small, mode):
    """The accumulate loops the large MSMs take, forced onto short and odd MSMs
    (ADVICE r4): k_msm_accumulate<true> (prefetching per-lane gathers) and
    k_msm_accumulate_coop (wave-cooperative LDS-DMA gathers, the 2^24 headline's
    loop: whole waves step together, lanes past the last entry feed row 0).
    Chunks shorter than the prefetch distance, bucket boundaries at a chunk's
    first entry (small scalars: few, crowded buckets), a partial last group and
    a partial last wave.  Bit-exact against the default loop of that size and
    against the trapdoor identity commit = [p(tau)] g."""
    import quill_amd as q
    rnd = random.Random(n * 7 + small)
    tau = rnd.randrange(R)
    scal = [rnd.randrange(1 << 12) if small else rnd.randrange(R) for _ in range(n)]
    d = q.Device(0)
    srs = q.Srs.generate(d, tau, n)
    out = {}
    for on in ("0", "1"):
        with env(mode, on), env("QG_MSM_COOP" if mode == "QG_MSM_PF" else "QG_MSM_PF", "0"):
            out[on] = srs.msm(scal)
    srs.close()
    d.close()
    assert out["0"] == out["1"]
    assert out["1"] == o.g1_mul(o.G1_GEN, o.poly_eval(scal, tau))


@pytest.mark.parametrize("nv", [9, 14, 17])
def test_side_stream_bucketing_matches_stream_order(dev, nv):
    """An ML opening runs its quotient MSMs as one batch whose 2nd.. MSMs bucket
    beside the previous MSM's accumulation, on two side streams by parity
    (msm_device_batch); QG_MSM_PIPE=0 keeps the batch on the context stream.
    Same proof and transcript state, and the opened value is the MLE
    evaluation."""
    import quill_amd as q
    from quill_amd import KZG, Transcript
    rnd = random.Random(4100 + nv)
    N = 1 << nv
    tau = rnd.randrange(R)
    kzg = KZG(dev, q.Srs.generate(dev, tau, N), N - 1)
    poly = [rnd.randrange(R) for _ in range(N)]
    vec = q.DeviceVec.from_list(dev, poly)
    point = [rnd.randrange(R) for _ in range(nv)]
    res = []
    for pipe in ("1", "0"):
        with env("QG_MSM_PIPE", pipe):
            t = Transcript(b"pipe")
            pr = kzg.open_dev(vec, N, point, t)
            res.append((pr, t.state))
    vec.close()
    kzg.srs.close()
    assert res[0] == res[1]
    assert res[0][0].evaluation == o.mle_evaluate(poly, point)


def test_open_batch_event_handover_matches_stream_order_and_oracle(dev):
    """The shape that failed in round 5 (profiles/r05_open_batch_ab.txt): one
    batched opening (qg_mle_open_batch_dev) of 10 vectors of 2^14..2^17
    entries, i.e. a 10-MSM S-commitment batch and a 40-MSM quotient batch on
    the two side streams, with event-ordered hand-overs (default), with
    host-synchronized hand-overs (QG_MSM_PIPE_SYNC=1) and in stream order
    (QG_MSM_PIPE=0), three times each, against successive single openings.
    Every proof field and the transcript state are identical, the oracle
    verifier (mlpcs.rs:126-161, KZG by the trapdoor identity) accepts every
    proof against [p(tau)] g, and the device hand-over guard never fired."""
    import oracle_c as oc
    from quill_amd import KZG, DeviceVec, Transcript
    tau = 0x48414E444F564552
    kzg = KZG.trusted_setup((1 << 17) - 1, tau, dev)
    rnd = random.Random(6060)
    # (log length, variables, live entries): full, zero-tailed (trims), a
    # public-column-like vector that trims to one entry, n > 2^nv, n < 2^nv
    shapes = [(17, 17, None), (16, 16, None), (17, 17, 5 << 14), (14, 14, None), (15, 15, None),
              (14, 14, 1), (16, 15, None), (15, 16, None), (17, 17, None), (14, 14, None)]
    vecs, arrs, items = [], [], []
    for k, (ln, nv, live) in enumerate(shapes):
        v = DeviceVec(dev, 1 << ln).fill_random(0x6060 + k)
        if live is not None:  # zero tail: the opening trims it (kzg.rs / ipa.rs)
            DeviceVec.from_u64(dev, np.zeros((1 << ln) - live, dtype=np.uint64), out=v, offset=live)
        vecs.append(v)
        arrs.append(v.to_numpy())
        items.append((v, 1 << ln, [rnd.randrange(R) for _ in range(nv)], False))
    items.append((vecs[0], 1 << 17, [rnd.randrange(R) for _ in range(17)], True))  # unchanged reuse
    ts = Transcript(b"handover")
    seq = [kzg.open_dev(v, n, pt, ts, unchanged=u) for v, n, pt, u in items]
    before = dev.counter("msm_handover_violation")
    for mode in ("events", "host", "stream") * 3:
        with env("QG_MSM_PIPE", "0" if mode == "stream" else "1"), \
                env("QG_MSM_PIPE_SYNC", "1" if mode == "host" else "0"):
            tb = Transcript(b"handover")
            got = kzg.open_batch_dev(items, tb)
        assert got == seq, mode
        assert tb.state == ts.state, mode
    assert dev.counter("msm_handover_violation") == before
    okzg = o.KZG((1 << 17) - 1, tau)
    vt = o.Transcript(b"handover")
    for (v, n, pt, _), proof in zip(items, seq):
        arr = arrs[vecs.index(v)]
        C = oc.g1_mul(o.G1_GEN, oc.fr_horner(arr, tau))
        pad = (1 << len(pt)) - len(arr)  # n < 2^nv: the zero-extended vector's MLE
        ext = np.vstack([arr, np.zeros((pad, 4), dtype=np.uint64)]) if pad > 0 else arr
        assert proof.evaluation == oc.fr_mle_eval(ext, pt)
        op = o.MLEvalProof(pt, proof.evaluation, proof.s_comm,
                           *[(getattr(proof, k).x, getattr(proof, k).y, getattr(proof, k).proof)
                             for k in ("poly_opening", "poly_opening_inv", "s_opening",
                                       "s_opening_inv")])
        assert op.verify(C, okzg, vt)
    assert vt.state == ts.state
    for v in vecs:
        v.close()
    kzg.close()


def test_hyperplonk_2p14_rows_event_handover_same_proof(dev):
    """HyperPlonk at 2^14 rows (the round-5 failing case, micro/open_batch_dbg.py):
    the proof with the MSM batches' event-ordered hand-overs equals, byte for
    byte, the proofs with host-synchronized hand-overs and in stream order;
    the oracle verifier accepts it; the hand-over guard never fired."""
    import hyperplonk_oracle as ho
    from quill_amd import KZG, HyperPlonk, serialize
    from quill_amd import examples as ex
    from test_gpu_hyperplonk import TAU, _oracle_setup, to_oracle
    rows = 1 << 14
    cws = [ex.fibonacci_circuit_and_trace(rows), ex.modified_fibonacci_circuit_and_trace(rows)]
    pcs = KZG.trusted_setup(max(c.num_cols() * c.num_rows() for c, _ in cws), TAU, dev)
    hp = HyperPlonk.preprocess([c for c, _ in cws], pcs)
    ws = [w for _, w in cws]
    before = dev.counter("msm_handover_violation")
    out = {}
    for mode in ("events", "host", "stream", "events"):
        with env("QG_MSM_PIPE", "0" if mode == "stream" else "1"), \
                env("QG_MSM_PIPE_SYNC", "1" if mode == "host" else "0"):
            proof = hp.prove(pcs, ws)
        enc = serialize(proof)
        assert out.setdefault(mode, enc) == enc, mode
        last = proof
    assert out["events"] == out["host"] == out["stream"]
    assert dev.counter("msm_handover_violation") == before
    opcs, ohp, _ = _oracle_setup(rows, ("fib", "mod"))
    vt = ho.hyperplonk_verify(to_oracle(last), ohp.to_vk(), opcs)
    assert vt.state == hp.last_transcript.state


def test_msm_dev_batch_equals_single_commits(dev):
    """qg_msm_g1_dev_batch (one MSM batch on the side streams) gives the same
    points as one qg_msm_g1_dev per vector: lengths 2^16, 1000, 0, 2^15 + 3 on
    one SRS, and the trapdoor identity [p(tau)] g for each."""
    import oracle_c as oc
    import quill_amd as q
    from quill_amd import KZG
    tau = 0x4241544348
    kzg = KZG.trusted_setup((1 << 16) - 1, tau, dev)
    vecs = [q.DeviceVec(dev, n).fill_random(77 + i) for i, n in enumerate((1 << 16, 1000, 1, (1 << 15) + 3))]
    ns = [1 << 16, 1000, 0, (1 << 15) + 3]
    got = kzg.srs.msm_dev_batch(vecs, ns)
    assert got == [kzg.srs.msm_dev(v, n) for v, n in zip(vecs, ns)]
    for v, n, P in zip(vecs, ns, got):
        want = oc.g1_mul(o.G1_GEN, oc.fr_horner(v.to_numpy(n), tau)) if n else None
        assert P == want
    assert kzg.commit_batch(vecs[:2]) == got[:2]
    for v in vecs:
        v.close()
    kzg.close()
