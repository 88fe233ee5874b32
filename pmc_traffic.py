"""HBM traffic of the bench kernels from rocprofv3 PMC counters.

Two separate counter passes (MI355X_MICROARCH.md, "rocprofv3 PMC slots": the
TCC block cannot hold FETCH_SIZE and WRITE_SIZE in one pass), each a child
`rocprofv3 --pmc X --kernel-trace -- python3 bench.py --traffic-probe ...`
started before the parent touches the GPU.  Corrections (same guide, "HBM"):
FETCH_SIZE / WRITE_SIZE are reported in KiB; on gfx950 FETCH_SIZE counts half
the bytes of wide streaming reads, so it is doubled; WRITE_SIZE is taken as is.
Per-launch bytes are returned for every kernel of the probe, with the achieved
HBM GB/s against the 8 TB/s peak from a third, kernel-trace-only pass (clean
per-launch durations)."""
from __future__ import annotations

import csv
import glob
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.abspath(__file__))
FETCH_FACTOR = 2 * 1024  # KiB -> B, x2 gfx950 FETCH_SIZE half-count
WRITE_FACTOR = 1024
# calibration launches of the probe (qg_microbench_fetch): CAL_GATHERS random
# 128-B row gathers from, then one streaming read of, a CAL_ROWS x 128-B table
# (8 GiB: far past the 256 MiB Infinity Cache)
CAL_ROWS = 1 << 26
CAL_GATHERS = 1 << 26
ROW_BYTES = 128


def _read_counters(outdir):
    rows = []
    for f in glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
    return rows


def _short(name):
    n = name.split("(")[0].replace("void ", "").strip()
    return n.split("::")[-1].split("<")[0]


# leg markers of the probe (bench.py traffic_probe: qg_trace_marker(tag), an
# empty kernel of `tag` 64-lane work-groups); profiles/kstats.py has the same map
MARKER = "k_trace_marker"
LEGS = {10: "probe_msm", 11: "probe_sumcheck", 12: "probe_logup", 13: "probe_mle",
        14: "probe_cal"}


def _leg_keys(rows):
    """[(row, leg)] for (dispatch, kernel, ..., grid work-items) rows in dispatch
    order, markers dropped: a dispatch belongs to the last marker's leg"""
    leg, out = "pre", []
    for r in sorted(rows, key=lambda r: r[0]):
        if r[1] == MARKER:
            tag = r[-1] // 64
            leg = LEGS.get(tag, f"tag{tag}")
            continue
        out.append((r, leg))
    return out


def kernel_durations(probe_args, timeout=300):
    """{kernel: (launches, average duration in us)} from a kernel-trace-only pass
    of the same probe (no counters: clean per-launch durations)"""
    exe = shutil.which("rocprofv3")
    if exe is None:
        raise RuntimeError("rocprofv3 not found")
    outdir = tempfile.mkdtemp(prefix="qg_kt_")
    try:
        cmd = [exe, "--kernel-trace", "-d", outdir, "-o", "kt", "-f", "csv", "--", sys.executable,
               os.path.join(ROOT, "bench.py"), "--traffic-probe"] + probe_args
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=timeout)
        if p.returncode != 0:
            raise RuntimeError(f"rocprofv3 --kernel-trace exited {p.returncode}: "
                               + p.stdout.decode(errors="replace")[-800:])
        acc, rows = {}, []
        for f in glob.glob(os.path.join(outdir, "**", "*kernel_trace.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                    rows.append((int(r.get("Dispatch_Id") or r["Start_Timestamp"]),
                                 _short(r["Kernel_Name"]), d, int(r["Grid_Size_X"])))
        for (_, k, d, g), leg in _leg_keys(rows):
            for key in (k, f"{k}@{g}", f"{k}#{leg}"):
                a = acc.setdefault(key, [0, 0.0])
                a[0] += 1
                a[1] += d
        return {k: (n, t / n) for k, (n, t) in acc.items()}
    finally:
        shutil.rmtree(outdir, ignore_errors=True)


def run_pass(counter, probe_args, timeout=300):
    """one rocprofv3 pass; `counter` is one name or a list that fits one pass
    (MI355X_MICROARCH.md "rocprofv3 PMC slots": <= 8 SQ, 4 TCC, 2 GRBM)"""
    counters = [counter] if isinstance(counter, str) else list(counter)
    exe = shutil.which("rocprofv3")
    if exe is None:
        raise RuntimeError("rocprofv3 not found")
    outdir = tempfile.mkdtemp(prefix="qg_pmc_")
    try:
        cmd = [exe, "--pmc"] + counters + ["--kernel-trace", "-d", outdir, "-o", "pmc", "-f",
                                           "csv", "--", sys.executable,
                                           os.path.join(ROOT, "bench.py"), "--traffic-probe"]
        cmd += probe_args
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=timeout)
        if p.returncode != 0:
            raise RuntimeError(f"rocprofv3 --pmc {counters} exited {p.returncode}: "
                               + p.stdout.decode(errors="replace")[-800:])
        rows = _read_counters(outdir)
        if not rows:
            raise RuntimeError(f"no counter rows for {counters}")
        if isinstance(counter, str):
            # (dispatch, kernel, value, grid work-items)
            return [(int(r["Dispatch_Id"]), _short(r["Kernel_Name"]), float(r["Counter_Value"]),
                     int(r.get("Grid_Size") or 0)) for r in rows if r["Counter_Name"] == counter]
        return [(int(r["Dispatch_Id"]), _short(r["Kernel_Name"]), r["Counter_Name"],
                 float(r["Counter_Value"])) for r in rows]
    finally:
        shutil.rmtree(outdir, ignore_errors=True)


def kernel_counters(passes, probe_args, timeout=300):
    """{kernel: {counter: value per launch}} over several passes (each a list)"""
    out = {}
    for counters in passes:
        rows = run_pass(list(counters), probe_args, timeout)
        launches = {}
        for did, k, name, v in rows:
            launches.setdefault(k, set()).add(did)
            d = out.setdefault(k, {})
            d[name] = d.get(name, 0.0) + v
        for k, ids in launches.items():
            for name in counters:
                if name in out[k]:
                    out[k][name] /= len(ids)
            out[k]["launches"] = len(ids)
    return out


def collect(probe_args, timeout=300):
    """{kernel: {"launches", "read_bytes_per_launch", "write_bytes_per_launch"}} plus
    the sumcheck per-call totals.  The probe runs one MSM then one sumcheck."""
    fetch = run_pass("FETCH_SIZE", probe_args, timeout)
    write = run_pass("WRITE_SIZE", probe_args, timeout)
    out = {}
    # per kernel, per kernel@grid (one launch shape = one problem size) and per
    # kernel#leg (the probe phase, from its markers)
    fetch_l, write_l = _leg_keys(fetch), _leg_keys(write)
    for rows, key, fac in ((fetch_l, "read_bytes", FETCH_FACTOR),
                           (write_l, "write_bytes", WRITE_FACTOR)):
        for (_, k, v, g), leg in rows:
            for kk in (k, f"{k}@{g}", f"{k}#{leg}"):
                d = out.setdefault(kk, {"launches": 0, "read_bytes": 0.0, "write_bytes": 0.0})
                d[key] += v * fac
    for (_, k, _, g), leg in fetch_l:
        for kk in (k, f"{k}@{g}", f"{k}#{leg}"):
            out[kk]["launches"] += 1
    for d in out.values():
        if "read_bytes" not in d:
            continue
        n = max(d["launches"], 1)
        d["read_bytes_per_launch"] = d.pop("read_bytes") / n
        d["write_bytes_per_launch"] = d.pop("write_bytes") / n
    # achieved HBM GB/s per kernel: PMC bytes per launch / clean average duration
    try:
        dur = kernel_durations(probe_args, timeout)
    except Exception as e:  # reported, never substituted
        dur = {}
        out["_duration_error"] = {"error": str(e)[-300:]}
    g, st = out.get("k_fetch_gather"), out.get("k_fetch_stream")
    if g and st and "read_bytes_per_launch" in g and "read_bytes_per_launch" in st:
        per_row = g["read_bytes_per_launch"] / CAL_GATHERS  # after the x2 correction
        out["_fetch_calibration"] = {
            "gather_rows": CAL_GATHERS, "table_bytes": CAL_ROWS * ROW_BYTES,
            "gather_corrected_bytes_per_row": per_row,
            "gather_read_factor": ROW_BYTES / per_row if per_row else None,
            "stream_corrected_over_true": st["read_bytes_per_launch"] / (CAL_ROWS * ROW_BYTES),
            "note": "corrected = FETCH_SIZE x2; stream_corrected_over_true ~1 confirms the x2 for "
                    "16-B-per-lane streams; gather_read_factor rescales reads so one random row "
                    "gather (five 16-B loads of a 128-B row, as msm_pt_load) counts 128 B"}
    for k, d in out.items():
        if k.startswith("_"):
            continue
        if k in dur and "read_bytes_per_launch" in d:
            us = dur[k][1]
            gbps = (d["read_bytes_per_launch"] + d["write_bytes_per_launch"]) / (us * 1e-6) / 1e9
            d["avg_us"] = us
            d["hbm_gbps"] = gbps
            d["frac_hbm_peak"] = gbps / HBM_PEAK_GBPS
    return out


HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


if __name__ == "__main__":
    # python pmc_traffic.py SQ_WAVES,SQ_INSTS_VALU GRBM_GUI_ACTIVE -- <bench.py probe args>
    import json
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    print(json.dumps(kernel_counters([a.split(",") for a in argv[:cut]], argv[cut + 1:]),
                     indent=1))
