"""Per-kernel HBM table from a bench.py JSON line (its `pmc` object: PMC bytes
per launch from FETCH_SIZE / WRITE_SIZE passes, clean durations from a
kernel-trace pass): achieved GB/s and fraction of the 8 TB/s HBM peak.
usage: python profiles/pmc_table.py <bench log or json> > profiles/<round>_kernel_hbm.txt"""
import json
import sys

line = [l for l in open(sys.argv[1]) if l.lstrip().startswith("{")][-1]
pmc = json.loads(line)["pmc"]
rows = [(k, d) for k, d in pmc.items() if isinstance(d, dict) and "hbm_gbps" in d and "@" in k]
rows.sort(key=lambda kv: -kv[1]["avg_us"] * kv[1]["launches"])
print("%-40s %8s %12s %12s %12s %10s %8s" % ("kernel", "launches", "avg_us", "read_MB", "write_MB",
                                             "GB/s", "frac"))
for k, d in rows:
    print("%-40s %8d %12.1f %12.1f %12.1f %10.1f %8.3f" % (
        k, d["launches"], d["avg_us"], d["read_bytes_per_launch"] / 1e6,
        d["write_bytes_per_launch"] / 1e6, d["hbm_gbps"], d["frac_hbm_peak"]))
