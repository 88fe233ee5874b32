"""qg_sumcheck_prove_cb: SumcheckProof::prove (sumcheck.rs:28-114) with the
caller's transcript authoritative through the challenge callback (SURVEY
8(b)).  A host transcript driven by the callback must give the proof, point,
evaluation and final transcript state of the device-transcript prove, bit for
bit; a failing callback aborts the prove."""
import random
import threading

import pytest

import quill_oracle as o

pytestmark = pytest.mark.gpu
R = o.R_MOD


def _exprs():
    from quill_amd import VirtualPolyExpr as E
    return {
        "product": E.Input(0) * E.Input(1) * E.Input(2),
        "mixed": E.Input(0) * E.Input(1) + E.Input(2) * E.Const(R - 5) + E.Const(7),
    }


def _callback_transcript(domain, nv, claimed):
    from quill_amd import Transcript
    t = Transcript(domain)
    t.append_u64(nv)  # sumcheck.rs:35-36, done by the caller in the callback form
    t.append_fr(claimed)

    def challenge(coeffs):
        t.append_poly(coeffs)  # sumcheck.rs:80
        return t.draw_field_element()  # sumcheck.rs:82
    return t, challenge


@pytest.mark.parametrize("kind,nv", [("product", 1), ("product", 11), ("mixed", 9)])
def test_callback_transcript_matches_device_transcript(dev, kind, nv):
    from quill_amd import DeviceVec, Transcript
    from quill_amd.hyperplonk import _unpack_dev, sumcheck_prove_callback, sumcheck_prove_device
    expr = _exprs()[kind]
    vecs = [DeviceVec(dev, 1 << nv).fill_random(0xCB0 + 3 * nv + i) for i in range(3)]
    claimed = random.Random(nv).randrange(R)
    t = Transcript(b"sumcheck_cb")
    want = _unpack_dev(nv, expr, *sumcheck_prove_device(dev, nv, vecs, expr, claimed, t))
    t2, challenge = _callback_transcript(b"sumcheck_cb", nv, claimed)
    got = sumcheck_prove_callback(dev, nv, vecs, expr, challenge)
    assert got == want
    assert t2.state == t.state
    for v in vecs:
        v.close()


def test_callback_failure_aborts(dev):
    from quill_amd import DeviceVec, VirtualPolyExpr as E
    from quill_amd.hyperplonk import sumcheck_prove_callback
    vecs = [DeviceVec(dev, 1 << 6).fill_random(0xCB1 + i) for i in range(2)]
    calls = []

    def challenge(coeffs):
        calls.append(len(coeffs))
        if len(calls) == 3:
            raise RuntimeError("transcript refused")
        return 12345

    with pytest.raises(RuntimeError, match="transcript refused"):
        sumcheck_prove_callback(dev, 6, vecs, E.Input(0) * E.Input(1), challenge)
    assert len(calls) == 3
    for v in vecs:
        v.close()


@pytest.mark.parametrize("world", [2, 4])
def test_callback_on_sharded_context(world):
    """every rank's own transcript replica through its callback: the sharded
    proof equals the single-context callback proof"""
    import quill_amd as q
    from quill_amd import DeviceVec
    from quill_amd.hyperplonk import sumcheck_prove_callback
    nv = 10
    expr = _exprs()["product"]
    rnd = random.Random(world)
    tabs = [[rnd.randrange(R) for _ in range(1 << nv)] for _ in range(3)]
    claimed = rnd.randrange(R)
    dev0 = q.Device(0)
    vecs = [DeviceVec.from_list(dev0, tb) for tb in tabs]
    t0, ch0 = _callback_transcript(b"sumcheck_cb_shard", nv, claimed)
    want = sumcheck_prove_callback(dev0, nv, vecs, expr, ch0)
    for v in vecs:
        v.close()
    dev0.close()
    group = q.Device.loopback_group(world)
    NL = (1 << nv) // world
    out, err = [None] * world, []

    def body(rank):
        try:
            d = q.Device(0)
            d.attach_loopback(group, rank)
            vs = [DeviceVec.from_list(d, tb[rank * NL:(rank + 1) * NL]) for tb in tabs]
            t, ch = _callback_transcript(b"sumcheck_cb_shard", nv, claimed)
            out[rank] = (sumcheck_prove_callback(d, nv, vs, expr, ch), t.state)
            for v in vs:
                v.close()
            d.close()
        except Exception as e:  # surfaced below
            err.append(e)
    ths = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=600)
    q.lib().qg_loopback_destroy(group)
    assert not err, err
    assert all(o_[0] == want and o_[1] == t0.state for o_ in out)
