"""BASELINE configs 4 and 5 in their SHARDED form at full size (VERDICT r4
"next" 1).  The multi-GPU rows exist for these two configs; their sharded code
had only run at 2^9 evaluations / 64 rows.

* C4: ML-PCS commit + open (MLEvalProof::prove, pcs/src/mlpcs.rs:83-124) of a
  2^22-evaluation vector, world 8 through the in-process loopback
  communicator (8 contexts on one GPU): eq table, inner product, the
  residue-split S polynomial at M = 2^22 (one all-to-all), the sharded
  quotient scans with their carry exchange, all six MSMs sharded.  Also one
  forced-RCCL run (QG_FORCE_RCCL=1: a real one-rank RCCL communicator, the
  sharded code path, ncclSend/ncclRecv for the all-to-all) at 2^22.
* C5: HyperPlonk::prove (hyperplonk/src/proof/proof.rs:239-301) of the
  fibonacci + modified-fibonacci traces (test_basic_proof.rs:17-105) at 2^20
  rows, world 8 loopback: the full-witness all-to-all, sharded zero-checks
  (early gather at nv 20), Logup columns, permutation checks, 26 openings.

Every rank's proof must equal the single-context proof byte for byte
(ark-serialize encoding, quill_amd/serialize.py) and end in the same transcript
state.  The single-context proofs are themselves pinned at these sizes by the
oracle verifiers (tests/test_gpu_headline.py).

Per-rank phase times (HIP events on each rank's stream; the 8 ranks share ONE
GPU here, so they are contended times, not an 8-GPU measurement) are written to
gpurun_out/sharded_full_times.json."""
import json
import os
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TIMES = os.path.join(ROOT, "gpurun_out", "sharded_full_times.json")
TAU = 0x5155494C4C2D53525321  # bench.py's synthetic trapdoor
PHASES = ("msm_bucketing", "msm_bucketing_side", "msm_accumulate", "msm_reduce", "sumcheck_round",
          "sumcheck_tail", "logup_column", "eq_table", "inner_product", "s_polynomial",
          "kzg_division")


def _record(key, value):
    os.makedirs(os.path.dirname(TIMES), exist_ok=True)
    data = {}
    if os.path.exists(TIMES):
        with open(TIMES) as f:
            data = json.load(f)
    data[key] = value
    with open(TIMES, "w") as f:
        json.dump(data, f, indent=1)


def _parts(dev):
    return {nm: round(dev.kernel_time(nm)[0], 3) for nm in PHASES if dev.kernel_time(nm)[1]}


def _run_ranks(world, fn):
    import quill_amd as q
    group = q.Device.loopback_group(world)
    out = [None] * world
    err = []

    def body(rank):
        dev = None
        try:
            dev = q.Device(0)
            dev.attach_loopback(group, rank)
            out[rank] = fn(dev, rank, world)
        except Exception as e:  # surfaced below
            err.append((rank, e))
        finally:
            if dev is not None:
                dev.close()

    ths = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=900)
    q.lib().qg_loopback_destroy(group)
    assert not err, err
    return out


def _mle_open(dev, srs, vec, L, n, k):
    """bench.py's C4 step: commit, absorb, draw the point, open"""
    from quill_amd import KZG, Transcript
    kzg = KZG(dev, srs, n - 1)
    C = srs.msm_dev(vec, L)
    t = Transcript(b"MLPCS full shard")
    t.append_g1(C)
    point = [t.draw_field_element() for _ in range(k)]
    pr = kzg.open_dev(vec, L, point, t)
    return C, pr, t.state


def _c4_single(k):
    import quill_amd as q
    n = 1 << k
    dev = q.Device(0)
    srs = q.Srs.generate(dev, TAU, n)
    vec = q.DeviceVec(dev, n).fill_random(0xC4C4 + k)
    host = vec.to_numpy()
    ref = _mle_open(dev, srs, vec, n, n, k)
    vec.close()
    srs.close()
    dev.close()
    return host, ref


def _upload_mont(dev, arr):
    import quill_amd as q
    from quill_amd._lib import check, lib
    from quill_amd.field import u64p
    arr = np.ascontiguousarray(arr, dtype=np.uint64)
    v = q.DeviceVec(dev, arr.shape[0])
    check(lib().qg_buf_upload(v.h, u64p(arr), arr.shape[0]), dev.h)
    return v


def test_c4_mle_open_2p22_world8_loopback_matches_single():
    import quill_amd as q
    k = 22
    n = 1 << k
    host, ref = _c4_single(k)

    def fn(dev, rank, world):
        L = n // world
        srs = q.Srs.generate(dev, TAU, L, offset=rank * L)
        vec = _upload_mont(dev, host[rank * L:(rank + 1) * L])
        _mle_open(dev, srs, vec, L, n, k)  # warm: scratch, twiddles, tables
        dev.enable_timing(True)
        t0 = time.perf_counter()
        res = _mle_open(dev, srs, vec, L, n, k)
        wall = time.perf_counter() - t0
        parts = _parts(dev)
        dev.enable_timing(False)
        vec.close()
        srs.close()
        return res, {"wall_ms": round(wall * 1e3, 3), "parts_ms": parts}

    outs = _run_ranks(8, fn)
    for (C, pr, st), _ in outs:
        assert C == ref[0]
        assert pr == ref[1]
        assert st == ref[2]
    _record("c4_mle_open_2p22_world8_loopback",
            {"what": "ML-PCS commit + open, 2^22 evaluations over 8 loopback ranks on one GPU "
                     "(contended per-rank times)",
             "ranks": [t for _, t in outs]})


def test_c4_mle_open_2p22_forced_rccl_matches_single():
    """world-1 sharded path over a real RCCL communicator at 2^22"""
    import quill_amd as q
    k = 22
    n = 1 << k
    host, ref = _c4_single(k)
    old = os.environ.get("QG_FORCE_RCCL")
    os.environ["QG_FORCE_RCCL"] = "1"
    try:
        rdev = q.Device(0)
        rdev.attach_comm(0, 1, q.Device.comm_unique_id())
    finally:
        if old is None:
            os.environ.pop("QG_FORCE_RCCL")
        else:
            os.environ["QG_FORCE_RCCL"] = old
    try:
        assert rdev.comm_info()["kind"] == "rccl" and rdev.comm_info()["sharded"]
        srs = q.Srs.generate(rdev, TAU, n)
        vec = _upload_mont(rdev, host)
        _mle_open(rdev, srs, vec, n, n, k)
        rdev.enable_timing(True)
        t0 = time.perf_counter()
        C, pr, st = _mle_open(rdev, srs, vec, n, n, k)
        wall = time.perf_counter() - t0
        parts = _parts(rdev)
        vec.close()
        srs.close()
    finally:
        rdev.close()
    assert (C, pr, st) == ref
    _record("c4_mle_open_2p22_forced_rccl_world1",
            {"what": "ML-PCS commit + open, 2^22, sharded path over a one-rank RCCL communicator",
             "wall_ms": round(wall * 1e3, 3), "parts_ms": parts})


def _c5_witnesses(rows):
    from quill_amd import examples as ex
    return [ex.fibonacci_circuit_and_trace(rows), ex.modified_fibonacci_circuit_and_trace(rows)]


def _c5_prove(dev, cws, timed=False):
    import quill_amd as q
    from quill_amd.serialize import serialize
    maxdeg = max(c.num_cols() * c.num_rows() for c, _ in cws)
    pcs = q.KZG.trusted_setup(maxdeg, TAU, dev)
    hp = q.HyperPlonk.preprocess([c for c, _ in cws], pcs)
    wits = [w for _, w in cws]
    info = None
    if timed:
        hp.prove(pcs, wits)  # warm: SRS shards, scratch, twiddles
        dev.enable_timing(True)
        t0 = time.perf_counter()
    proof = hp.prove(pcs, wits)
    if timed:
        info = {"wall_ms": round((time.perf_counter() - t0) * 1e3, 3), "parts_ms": _parts(dev)}
        dev.enable_timing(False)
    vks = [(vk.public_columns_commitments, vk.id_commitment, vk.permutation_commitment)
           for vk in hp.trace_vks]
    out = (serialize(proof), hp.last_transcript.state, vks)
    for pk in hp.trace_pks:
        for v in [pk.id_poly, pk.permutation_poly] + pk.public_values + pk.public_rows:
            v.close()
    pcs.close()
    return out, info


def test_c5_hyperplonk_2p20_rows_world8_loopback_matches_single():
    import quill_amd as q
    rows = 1 << 20
    cws = _c5_witnesses(rows)
    dev0 = q.Device(0)
    ref, _ = _c5_prove(dev0, cws)
    dev0.close()

    outs = _run_ranks(8, lambda dev, rank, world: _c5_prove(dev, cws, timed=True))
    for (pbytes, state, vks), _ in outs:
        assert vks == ref[2]
        assert state == ref[1]
        assert pbytes == ref[0]
    _record("c5_hyperplonk_2p20_rows_world8_loopback",
            {"what": "HyperPlonk prove, fib + mod-fib at 2^20 rows over 8 loopback ranks on one "
                     "GPU (contended per-rank times)",
             "proof_bytes": len(ref[0]), "ranks": [t for _, t in outs]})
