"""Logup column timing for library A/B runs (QG_LIB selects the build): the
bench's logup workload (m / (beta + t0 + a t1), 2^k rows), kernel time from the
library's events and the column sum, so builds can be compared for equality.

usage: QG_LIB=... python micro/logup_prof.py [log_rows] [calls]
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
from quill_amd import VirtualPolyExpr as E  # noqa: E402
from quill_amd.logup import logup_column_device  # noqa: E402
from bench import LOGUP_A, LOGUP_BETA  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = q.Device(0)
    n = 1 << k
    tabs = [q.DeviceVec(dev, n).fill_random(0x5155494C4C + 5 + 11 * i) for i in range(3)]
    out = q.DeviceVec(dev, n)
    h = E.Input(0) + E.Const(LOGUP_A) * E.Input(1)
    m = E.Input(2)
    s = logup_column_device(dev, k, tabs, h, LOGUP_BETA, out, m)
    dev.enable_timing(True)
    t0 = time.perf_counter()
    for _ in range(calls):
        s = logup_column_device(dev, k, tabs, h, LOGUP_BETA, out, m)
    dt = (time.perf_counter() - t0) / calls
    kms, _ = dev.kernel_time("logup_column")
    print(f"2^{k} rows: {dt * 1e3:.4f} ms/call  kernels {kms / calls:.4f} ms  "
          f"sum_low64 {s & ((1 << 64) - 1):#x}", flush=True)
    for t in tabs + [out]:
        t.close()
    dev.close()


if __name__ == "__main__":
    main()
