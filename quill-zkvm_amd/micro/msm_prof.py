"""MSM kernel profile driver (run under rocprofv3 --kernel-trace --stats):
one SRS of 2^max bases, then `reps` MSMs at each requested size, each result
checked against the trapdoor identity with the oracle's C Horner.

usage: python micro/msm_prof.py [log_max] [log_sizes,comma-separated] [reps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "quill-zkvm_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

if os.environ.get("QG_LIB"):  # A/B builds of the library (micro benchmark only)
    import quill_amd._lib as _L  # noqa: E402
    _L.LIB_PATH = os.path.abspath(os.environ["QG_LIB"])
import quill_amd as q  # noqa: E402
import oracle_c as oc  # noqa: E402

TAU = 0x5155494C4C2D53525321


def main():
    lmax = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    sizes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [lmax]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    dev = q.Device(0)
    own = os.environ.get("MSM_PROF_OWN_SRS") == "1"  # an SRS per size (its own window bits)
    srs = None if own else q.Srs.generate(dev, TAU, 1 << lmax)
    scalars = q.DeviceVec(dev, 1 << lmax).fill_random(0x5155494C4C + 2)
    oc.lib()
    for lg in sizes:
        n = 1 << lg
        if own:
            if srs is not None:
                srs.close()
            srs = q.Srs.generate(dev, TAU, n)
        srs.msm_dev(scalars, n)  # warm
        dev.enable_timing(True)
        t0 = time.perf_counter()
        for _ in range(reps):
            res = srs.msm_dev(scalars, n)
        dt = (time.perf_counter() - t0) / reps
        parts = {nm: dev.kernel_time(nm)[0] / reps for nm in
                 ("msm_bucketing", "msm_accumulate", "msm_reduce")}
        dev.enable_timing(False)
        v = oc.fr_horner(scalars.to_numpy(n), TAU)
        ok = oc.g1_mul((1, 2), v) == res
        print(f"2^{lg}: {dt * 1e3:.3f} ms/msm  c={srs.window_info()[0]}  " +
              "  ".join(f"{k} {v:.3f}" for k, v in parts.items()) + f"  verified={ok}",
              flush=True)
        assert ok or os.environ.get("MSM_PROF_NOCHECK") == "1"  # timing-only experiment builds
    srs.close()
    scalars.close()
    dev.close()


if __name__ == "__main__":
    main()
