"""HyperPlonk proofs at 2^k rows under QUILL_OPEN_BATCH / QG_MSM_PIPE
combinations, compared opening by opening (debug driver).
usage: python micro/open_batch_dbg.py [log_rows]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "quill-zkvm_amd"))
import quill_amd as q  # noqa: E402
from quill_amd import KZG, HyperPlonk  # noqa: E402
from quill_amd import examples as ex  # noqa: E402

TAU = 0x5155494C4C2D53525321


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 14
    rows = 1 << k
    dev = q.Device(0)
    cws = [ex.fibonacci_circuit_and_trace(rows), ex.modified_fibonacci_circuit_and_trace(rows)]
    maxdeg = max(c.num_cols() * c.num_rows() for c, _ in cws)
    pcs = KZG.trusted_setup(maxdeg, TAU, dev)
    hp = HyperPlonk.preprocess([c for c, _ in cws], pcs)
    ws = [w for _, w in cws]
    res = {}
    for batch, pipe, sp in (("0", "0", "0"), ("1", "1", "0"), ("0", "1", "0")):
        os.environ["QUILL_OPEN_BATCH"] = batch
        os.environ["QG_MSM_PIPE"] = pipe
        os.environ["QG_MSM_SYNC_PLAN"] = sp
        pr = hp.prove(pcs, ws)
        res[(batch, pipe, sp)] = (pr, hp.last_transcript.state)
    ref, ref_state = res[("0", "0", "0")]
    for key, (pr, st) in res.items():
        print(key, "state equal:", st == ref_state, flush=True)
        for ti, (a, b) in enumerate(zip(pr.trace_proofs, ref.trace_proofs)):
            names = ["zc%d" % i for i in range(len(a.openings_zero_check))] + \
                    ["pub%d" % i for i in range(len(a.openings_public))] + ["id", "perm", "pt"]
            oa = list(a.openings_zero_check) + list(a.openings_public) + \
                [a.opening_id, a.opening_permutation, a.opening_permutation_trace]
            ob = list(b.openings_zero_check) + list(b.openings_public) + \
                [b.opening_id, b.opening_permutation, b.opening_permutation_trace]
            for nm, x, y in zip(names, oa, ob):
                if x != y:
                    diffs = [f for f in ("evaluation", "s_comm", "poly_opening", "poly_opening_inv",
                                         "s_opening", "s_opening_inv")
                             if getattr(x, f) != getattr(y, f)]
                    print("  trace", ti, nm, "differs:", diffs, flush=True)
    dev.close()


if __name__ == "__main__":
    main()
