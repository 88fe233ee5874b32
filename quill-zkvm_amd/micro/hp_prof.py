"""HyperPlonk prove timing for library A/B runs (bench.py's hyperplonk leg
without the rest of the bench): one warm proof, then `steps` timed proofs,
phase times from the library's HIP-event timers, and the final transcript
state (identical across variants when the proof is).

usage: QG_LIB=... python micro/hp_prof.py [log_rows] [steps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "quill-zkvm_amd"))
sys.path.insert(0, ROOT)

if os.environ.get("QG_LIB"):  # A/B builds of the library (micro benchmark only)
    import quill_amd._lib as _L  # noqa: E402
    _L.LIB_PATH = os.path.abspath(os.environ["QG_LIB"])
import quill_amd as q  # noqa: E402
from quill_amd import KZG, HyperPlonk, TraceWitness  # noqa: E402
from quill_amd import examples as ex  # noqa: E402
from bench import HP_PHASES, TAU  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = q.Device(0)
    rows = 1 << k
    cws = [ex.fibonacci_circuit_and_trace(rows), ex.modified_fibonacci_circuit_and_trace(rows)]
    maxdeg = max(c.num_cols() * c.num_rows() for c, _ in cws)
    pcs = KZG.trusted_setup(maxdeg, TAU, dev)
    hp = HyperPlonk.preprocess([c for c, _ in cws], pcs)
    wits = []
    for c, w in cws:
        buf = q.DeviceVec(dev, rows * c.num_cols())
        for i, col in enumerate(w):
            q.DeviceVec.from_canonical(dev, col, out=buf, offset=i * rows)
        wits.append(TraceWitness.from_full(buf, c.num_cols()))
    hp.prove(pcs, wits)
    if os.environ.get("HP_PROF_CPROFILE") == "1":  # host-side profile of the timed proofs
        import cProfile
        import pstats
        pr = cProfile.Profile()
        t0 = time.perf_counter()
        pr.enable()
        for _ in range(steps):
            hp.prove(pcs, wits)
        pr.disable()
        print(f"2^{k}: {(time.perf_counter() - t0) / steps * 1e3:.1f} ms/proof under cProfile")
        st = pstats.Stats(pr)
        st.sort_stats("tottime").print_stats(35)
        st.sort_stats("cumtime").print_stats(35)
        return
    dev.enable_timing(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        hp.prove(pcs, wits)
    dt = (time.perf_counter() - t0) / steps
    parts = {nm: round(dev.kernel_time(nm)[0] / steps, 2) for nm in HP_PHASES}
    print(f"2^{k}: {dt * 1e3:.1f} ms/proof  {parts}  state={hp.last_transcript.state.hex()[:16]}",
          flush=True)


if __name__ == "__main__":
    main()
