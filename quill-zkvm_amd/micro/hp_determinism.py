"""Repeat the 2^14-row HyperPlonk prove (fib + mod-fib, tests/test_gpu_hyperplonk.py)
R times in one process and compare every opening's fields with run 0, and
verify each run with the oracle verifier: finds nondeterministic proofs and
names the first opening / field that differs.

usage: python micro/hp_determinism.py [rows_log] [runs]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "quill-zkvm_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import quill_amd as q  # noqa: E402
import hyperplonk_oracle as ho  # noqa: E402
from test_gpu_hyperplonk import _device_setup, _oracle_setup, to_oracle  # noqa: E402

FIELDS = ("poly_opening", "poly_opening_inv", "s_opening", "s_opening_inv")


def flat(proof):
    out = []
    for t, tp in enumerate(proof.trace_proofs):
        ops = ([("zc%d" % i, o) for i, o in enumerate(tp.openings_zero_check)]
               + [("pub%d" % i, o) for i, o in enumerate(tp.openings_public)]
               + [("id", tp.opening_id), ("perm", tp.opening_permutation),
                  ("pt", tp.opening_permutation_trace)])
        for name, o in ops:
            out.append((f"t{t}.{name}.eval", o.evaluation))
            out.append((f"t{t}.{name}.s_comm", o.s_comm))
            for k in FIELDS:
                op = getattr(o, k)
                out.append((f"t{t}.{name}.{k}", (op.x, op.y, op.proof)))
    return out


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 14
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    dev = q.Device(0)
    pcs, hp, ws = _device_setup(dev, 1 << k, ("fib", "mod"))
    opcs, ohp, _ = _oracle_setup(1 << k, ("fib", "mod"))
    ref = None
    for r in range(runs):
        proof = hp.prove(pcs, ws)
        f = flat(proof)
        ok = True
        try:
            ho.hyperplonk_verify(to_oracle(proof), ohp.to_vk(), opcs)
        except ValueError as e:
            ok = f"verify failed: {e}"
        diffs = [] if ref is None else [a[0] for a, b in zip(f, ref) if a[1] != b[1]]
        print(f"run {r}: verify={ok} state={hp.last_transcript.state.hex()[:16]} "
              f"diffs={len(diffs)} first={diffs[:6]}", flush=True)
        if ref is None:
            ref = f


if __name__ == "__main__":
    main()
