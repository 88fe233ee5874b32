"""Per-kernel HBM table from bench.py's PMC probe (the `pmc` object of the
--detail-out JSON, or of a bench log's JSON line): PMC bytes per launch
(FETCH_SIZE x2 KiB-corrected + WRITE_SIZE, separate passes), clean average
duration from a kernel-trace-only pass, achieved GB/s and fraction of the
8 TB/s HBM peak.  Rows are kernel#leg (the probe phase from its
qg_trace_marker markers: probe_msm = the 2^log-msm headline MSM,
probe_sumcheck, probe_logup, probe_mle) with the launch shape beside them.
usage: python profiles/pmc_table.py <bench_detail.json | bench log> [--shapes]"""
import json
import sys


def load(path):
    txt = open(path).read()
    try:
        d = json.loads(txt)
    except json.JSONDecodeError:
        d = json.loads([ln for ln in txt.splitlines() if ln.lstrip().startswith("{")][-1])
    return d["pmc"]


def main():
    pmc = load(sys.argv[1])
    sep = "@" if "--shapes" in sys.argv else "#"
    rows = [(k, d) for k, d in pmc.items()
            if isinstance(d, dict) and "hbm_gbps" in d and sep in k]
    rows.sort(key=lambda kv: -kv[1]["avg_us"] * kv[1]["launches"])
    print("%-44s %8s %11s %11s %11s %9s %7s" % ("kernel" + sep + ("grid" if sep == "@" else "leg"),
                                                 "launches", "avg_us", "read_MB", "write_MB",
                                                 "GB/s", "frac"))
    for k, d in rows:
        print("%-44s %8d %11.1f %11.2f %11.2f %9.1f %7.4f" % (
            k, d["launches"], d["avg_us"], d["read_bytes_per_launch"] / 1e6,
            d["write_bytes_per_launch"] / 1e6, d["hbm_gbps"], d["frac_hbm_peak"]))
    cal = pmc.get("_fetch_calibration")
    if cal:
        print("\nFETCH_SIZE calibration: stream corrected/true = %.3f, random 128-B row gather "
              "corrected bytes/row = %.1f" % (cal["stream_corrected_over_true"],
                                              cal["gather_corrected_bytes_per_row"]))


if __name__ == "__main__":
    main()
