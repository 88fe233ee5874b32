"""FETCH_SIZE of random 128-B row gathers vs table size (micro benchmark, not a
test): python fetch_cal.py <log2 rows> <log2 gathers>; run under
rocprofv3 --pmc FETCH_SIZE --kernel-trace."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import quill_amd as q  # noqa: E402

lr, lg = int(sys.argv[1]), int(sys.argv[2])
dev = q.Device(0)
g, s = dev.microbench_fetch(1 << lr, 1 << lg)
print(f"rows 2^{lr} ({(128 << lr) / 2**30:.1f} GiB) gathers 2^{lg}: gather {g:.3f} ms "
      f"({(1 << lg) * 128 / g / 1e6:.0f} GB/s at 128 B/row), stream {s:.3f} ms")
