"""HyperPlonk 2^k-row proofs in one process under a sequence of MSM-batch
hand-over modes (events = event-ordered, host = host synchronizations,
stream = QG_MSM_PIPE=0), each compared opening by opening with run 0 and
verified by the oracle verifier; prints the hand-over guard counter.

usage: python micro/handover_dbg.py [rows_log] [mode,mode,...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "quill-zkvm_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "quill-zkvm_amd", "micro"))

import quill_amd as q  # noqa: E402
import hyperplonk_oracle as ho  # noqa: E402
from test_gpu_hyperplonk import _device_setup, _oracle_setup, to_oracle  # noqa: E402
from hp_determinism import flat  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 14
    modes = (sys.argv[2] if len(sys.argv) > 2 else "events,events,host,host,stream,stream,events").split(",")
    dev = q.Device(0)
    pcs, hp, ws = _device_setup(dev, 1 << k, ("fib", "mod"))
    opcs, ohp, _ = _oracle_setup(1 << k, ("fib", "mod"))
    ref = None
    for r, mode in enumerate(modes):
        os.environ["QG_MSM_PIPE"] = "0" if mode == "stream" else "1"
        os.environ["QG_MSM_PIPE_SYNC"] = "1" if mode == "host" else "0"
        os.environ["QUILL_OPEN_BATCH"] = "0" if mode == "seq" else "1"
        proof = hp.prove(pcs, ws)
        f = flat(proof)
        ok = True
        try:
            ho.hyperplonk_verify(to_oracle(proof), ohp.to_vk(), opcs)
        except ValueError as e:
            ok = f"FAILED: {e}"
        diffs = [] if ref is None else [a[0] for a, b in zip(f, ref) if a[1] != b[1]]
        print(f"run {r} {mode}: verify={ok} state={hp.last_transcript.state.hex()[:16]} "
              f"diffs={len(diffs)} first={diffs[:8]} guard={dev.counter('msm_handover_violation')}",
              flush=True)
        if ref is None:
            ref = f
    dev.close()


if __name__ == "__main__":
    main()
