"""S-polynomial cost per rank of a sharded ML opening (micro benchmark, not a
test): MLEvalProof::prove at 2^k evaluations over W in-process loopback ranks
on ONE GPU, per-rank device time of the "s_polynomial" kernel group (HIP
events on each rank's stream).  The ranks share the device, so the sum over
ranks is the GPU work of the whole job; its ratio to the single-context time
is what W real GPUs would divide.  Run once as is (residue split) and once
with QG_S_REPLICATED=1 (the whole S on every rank).
usage: python spoly_ab.py <log2 evals> <W>..."""
import json
import os
import sys
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
if os.environ.get("QG_LIB"):  # A/B builds of the library (micro benchmark only)
    import quill_amd._lib as _L  # noqa: E402
    _L.LIB_PATH = os.path.abspath(os.environ["QG_LIB"])
import quill_amd as q  # noqa: E402
from quill_amd import KZG, Transcript  # noqa: E402

k = int(sys.argv[1])
worlds = [int(x) for x in sys.argv[2:]] or [1, 2, 4, 8]
N = 1 << k
TAU = 0x5155494C4C2D53525321
out = {"log_evals": k, "replicated": bool(os.environ.get("QG_S_REPLICATED")), "runs": []}
for W in worlds:
    L = N // W
    group = q.Device.loopback_group(W) if W > 1 else None
    res = [None] * W
    errs = []

    def body(rank):
        try:
            dev = q.Device(0)
            if group is not None:
                dev.attach_loopback(group, rank)
            kzg = KZG(dev, q.Srs.generate(dev, TAU, L, offset=rank * L), N - 1)
            poly = q.DeviceVec(dev, L).fill_random(0x5155494C4C + 4 + 1000 * rank)
            pt = [(7 * i + 3) % 1000003 for i in range(k)]
            kzg.open_dev(poly, L, pt, Transcript(b"spoly"))  # warm-up (twiddles, scratch)
            dev.enable_timing(True)
            kzg.open_dev(poly, L, pt, Transcript(b"spoly"))
            res[rank] = dev.kernel_time("s_polynomial")[0]
            dev.enable_timing(False)
            poly.close()
            kzg.srs.close()
            dev.close()
        except Exception as e:  # reported
            errs.append(repr(e))

    ths = [threading.Thread(target=body, args=(r,)) for r in range(W)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=600)
    if group is not None:
        q.lib().qg_loopback_destroy(group)
    out["runs"].append({"world": W, "s_poly_ms_per_rank": res, "sum_ms": sum(x or 0 for x in res),
                        "max_ms": max(x or 0 for x in res), "errors": errs})
print(json.dumps(out))
