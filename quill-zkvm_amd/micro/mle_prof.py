"""ML-PCS commit + open timing for library A/B runs (bench.py's mle_open leg
without the rest of the bench; QG_LIB selects the build): one warm step, then
`steps` timed ones; prints the wall time per step and a digest of the last
proof and transcript state (identical across builds when the proofs are).

usage: QG_LIB=... python micro/mle_prof.py [log_evals] [steps]
"""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "quill-zkvm_amd"))

if os.environ.get("QG_LIB"):  # A/B builds of the library (micro benchmark only)
    import quill_amd._lib as _L  # noqa: E402
    _L.LIB_PATH = os.path.abspath(os.environ["QG_LIB"])
import quill_amd as q  # noqa: E402
from quill_amd import KZG, Transcript  # noqa: E402

TAU = 0x5155494C4C2D53525321


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = q.Device(0)
    n = 1 << k
    kzg = KZG(dev, q.Srs.generate(dev, TAU, n), n - 1)
    poly = q.DeviceVec(dev, n).fill_random(0x5155494C4C + 4)

    def step():
        C = kzg.srs.msm_dev(poly)
        t = Transcript(b"MLPCS bench")
        t.append_g1(C)
        point = [t.draw_field_element() for _ in range(k)]
        return kzg.open_dev(poly, n, point, t), t

    step()
    t0 = time.perf_counter()
    for _ in range(steps):
        proof, t = step()
    dt = (time.perf_counter() - t0) / steps
    digest = hashlib.sha256(repr(proof).encode() + t.state).hexdigest()[:16]
    print(f"2^{k}: {dt * 1e3:.3f} ms/step  proof+state {digest}", flush=True)


if __name__ == "__main__":
    main()
