"""Phase timeline of one 2^n sumcheck prove (micro benchmark, not a test):
loads micro/libquill_gpu_trace.so (make -C quill-zkvm_amd trace) and prints
per-round phase durations from the device timestamps (100 MHz clock)."""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import quill_amd._lib as L  # noqa: E402

L.LIB_PATH = os.path.join(HERE, "libquill_gpu_trace.so")
import quill_amd as q  # noqa: E402
from quill_amd.hyperplonk import VirtualPolyExpr as E, sumcheck_prove_device  # noqa: E402

nv = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = q.Device(0)
tabs = [q.DeviceVec(dev, 1 << nv).fill_random(11 + i) for i in range(3)]
expr = E.Input(0) * E.Input(1) * E.Input(2)
for _ in range(3):
    sumcheck_prove_device(dev, nv, tabs, expr, 0, q.Transcript(b"t"))
lib = L.lib()
fn = lib.qg_debug_sc_trace
fn.argtypes = [C.POINTER(C.c_uint64), C.c_size_t]
NB = 2048 + 4 * 1536
buf = (C.c_uint64 * NB)()
fn(buf, NB)
tick = 0.01  # us per 100 MHz tick
names_r = ["start", "evaluated(b0)", "last-block", "interp", "hash1", "hash2", "chal", "end"]
print("round kernels (block 0 / last block), us relative to kernel start")
for j in range(nv):
    b = 1024 + 16 * j
    if buf[b] == 0 or buf[b + 7] == 0:
        continue
    t0 = buf[b]
    print(j, " ".join(f"{names_r[k]}={(buf[b + k] - t0) * tick:.2f}" for k in range(1, 8)
                      if buf[b + k]), f"rows-summed={(buf[b + 8] - t0) * tick:.2f}" if buf[b + 8] else "")
names_t = ["start", "evaluated", "reduced", "interp", "hash1", "hash2", "chal", "blockred", "barrier"]
print("tail rounds, us relative to round start")
for j in range(nv):
    b = 16 * j
    if buf[b] == 0 or buf[b + 6] == 0:
        continue
    t0 = buf[b]
    print(j, " ".join(f"{names_t[k]}={(buf[b + k] - t0) * tick:.2f}" for k in (1, 7, 8, 2, 3, 4, 5, 6)
                      if buf[b + k] >= t0))
print("big rounds, per block: start / sweep-end spread (us from the earliest block start)")
for j in range(4):
    base = 2048 + j * 1536
    rows = [(buf[base + 3 * b], buf[base + 3 * b + 1], buf[base + 3 * b + 2]) for b in range(512)]
    rows = [(b, s0, e, cu) for b, (s0, e, cu) in enumerate(rows) if s0 and e]
    if not rows:
        continue
    t0 = min(s0 for _, s0, _, _ in rows)
    st = sorted((s0 - t0) * tick for _, s0, _, _ in rows)
    en = sorted((e - t0) * tick for _, _, e, _ in rows)
    du = sorted((e - s0) * tick for _, s0, e, _ in rows)
    q = lambda v: " ".join(f"{v[int(f * (len(v) - 1))]:.1f}" for f in (0, .1, .5, .9, 1))
    print(f"round {j}: blocks={len(rows)} start[min p10 p50 p90 max]={q(st)} end={q(en)} dur={q(du)}")
    cus = {}
    for b, s0, e, cu in rows:
        cus.setdefault(cu, []).append(b)
    per = sorted(len(v) for v in cus.values())
    print(f"  distinct CU ids={len(cus)} blocks per CU id min/max={per[0]}/{per[-1]}")
    slow = sorted(rows, key=lambda r: r[2] - r[1])[-5:]
    fast = sorted(rows, key=lambda r: r[2] - r[1])[:5]
    print("  fastest (block, dur us, cu)", [(b, round((e - s0) * tick, 1), cu) for b, s0, e, cu in fast])
    print("  slowest (block, dur us, cu)", [(b, round((e - s0) * tick, 1), cu) for b, s0, e, cu in slow])
