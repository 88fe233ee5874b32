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
