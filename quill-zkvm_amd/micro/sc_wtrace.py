"""Per-wave sweep end times of the big sumcheck rounds (micro benchmark, not a
test): loads micro/libquill_gpu_trace.so and groups the waves of every round by
(CU, SIMD) from the HW_ID register, to see whether waves sit unevenly on the
SIMDs of a CU and whether the crowded SIMDs are the late ones."""
import collections
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
NB = 2048 + 4 * 1536
buf = (C.c_uint64 * NB)()
lib.qg_debug_sc_trace.argtypes = [C.POINTER(C.c_uint64), C.c_size_t]
lib.qg_debug_sc_trace(buf, NB)
NW = 4 * 512 * 8 * 2
wb = (C.c_uint64 * NW)()
lib.qg_debug_sc_wtrace.argtypes = [C.POINTER(C.c_uint64), C.c_size_t]
lib.qg_debug_sc_wtrace(wb, NW)
tick = 0.01
for j in range(4):
    base = 2048 + j * 1536
    blocks = {}
    for b in range(512):
        s0, cu = buf[base + 3 * b], buf[base + 3 * b + 2]
        if s0:
            blocks[b] = (s0, cu)
    if not blocks:
        continue
    t0 = min(s for s, _ in blocks.values())
    waves = []
    for b, (s0, cu) in blocks.items():
        for w in range(8):
            o = ((j * 512 + b) * 8 + w) * 2
            if wb[o] >= s0 and wb[o]:
                hw = wb[o + 1]
                waves.append((b, w, cu, (hw >> 4) & 3, (wb[o] - t0) * tick))
    per = collections.defaultdict(list)
    for b, w, cu, simd, e in waves:
        per[(cu, simd)].append(e)
    hist = collections.Counter(len(v) for v in per.values())
    print(f"round {j}: waves={len(waves)} (CU,SIMD) pairs={len(per)} waves-per-SIMD histogram={dict(sorted(hist.items()))}")
    by = collections.defaultdict(list)
    for v in per.values():
        by[len(v)].extend(v)
    for n, v in sorted(by.items()):
        v.sort()
        print(f"  SIMDs holding {n} wave(s): end us min/p50/max = {v[0]:.1f} / {v[len(v) // 2]:.1f} / {v[-1]:.1f}")
    xw = collections.defaultdict(list)
    for b, w, cu, simd, e in waves:
        xw[wb[((j * 512 + b) * 8 + w) * 2 + 1] >> 32].append(e)
    for x, v in sorted(xw.items()):
        v.sort()
        print(f"  XCC {x}: waves={len(v)} end us min/p50/max = {v[0]:.1f} / {v[len(v) // 2]:.1f} / {v[-1]:.1f}")
    cuw = collections.Counter(cu for _, _, cu, _, _ in waves)
    print(f"  waves per CU min/max = {min(cuw.values())}/{max(cuw.values())}")
