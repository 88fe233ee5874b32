"""C5 CPU baseline at 2^12 rows (>= 2^12), timed on the GPU box's
host: python quill-zkvm_amd/micro/hp_cpu12.py [log_rows]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import hyperplonk_c as hc  # noqa: E402
import hyperplonk_oracle as ho  # noqa: E402
import quill_oracle as qo  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 12
rows = 1 << lg
TAU = 0x5155494C4C2D53525321
c1, w1 = ho.fibonacci_circuit_and_trace(rows)
c2, w2 = ho.modified_fibonacci_circuit_and_trace(rows)
pcs = qo.KZG(max(c1.num_cols(), c2.num_cols()) * rows, TAU)
hp = ho.HyperPlonk.preprocess([c1, c2], pcs)
with hc.c_backend(TAU, pcs.max_degree + 1):
    t0 = time.perf_counter()
    proof, t = hp.prove(pcs, [w1, w2])
    sec = time.perf_counter() - t0
print(f'{{"log_rows": {lg}, "seconds": {sec:.3f}, "cores": 1, "final_state": "{t.state.hex()}"}}',
      flush=True)
