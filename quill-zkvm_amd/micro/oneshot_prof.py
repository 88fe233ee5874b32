"""One-shot-bases MSM timing (qg_bases_upload) against the window-shifted SRS
path on the same bases and scalars: upload (one table) time, MSM ms, equality.
usage: python micro/oneshot_prof.py [logn] [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import quill_amd as q  # noqa: E402
from quill_amd import Srs  # noqa: E402

logn = int(sys.argv[1]) if len(sys.argv) > 1 else 24
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
n = 1 << logn
dev = q.Device(0)
t0 = time.perf_counter()
full = Srs.generate(dev, 0x5EED + logn, n)
t_gen = time.perf_counter() - t0
xy, inf = full.download_raw()
t0 = time.perf_counter()
one = Srs.upload_raw(dev, xy, inf, oneshot=True)
t_one = time.perf_counter() - t0
t0 = time.perf_counter()
tab = Srs.upload_raw(dev, xy, inf, oneshot=False)
t_tab = time.perf_counter() - t0
tab.close()
v = q.DeviceVec(dev, n).fill_random(4242)
ref = full.msm_dev(v, n)
res = {}
for name, s in (("oneshot", one), ("srs_tables", full)):
    s.msm_dev(v, n)
    dev.synchronize() if hasattr(dev, "synchronize") else None
    t0 = time.perf_counter()
    for _ in range(steps):
        got = s.msm_dev(v, n)
    res[name + "_ms"] = (time.perf_counter() - t0) / steps * 1e3
    res[name + "_equal"] = got == ref
print(json.dumps({"logn": logn, "steps": steps, "srs_generate_s": t_gen,
                  "upload_oneshot_s": t_one, "upload_with_tables_s": t_tab, **res}))
v.close()
one.close()
full.close()
