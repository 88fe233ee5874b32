"""Per-kernel summary (launch shape, count, average/total us, VGPRs, scratch)
of a rocprofv3 SQLite output (ROCm 7 rocpd format):

  python profiles/kstats.py <dir-or-db> [name-substring] [--legs]

--legs: every dispatch is attributed to the bench leg it ran in.  bench.py
launches an empty `k_trace_marker` of `tag` work-groups (64 work-items each) at
the start of each leg (qg_trace_marker); a dispatch belongs to the leg of the
last marker before it on the same process, so launches of one kernel with the
same grid in different legs (the 2^24 headline accumulate and the 2^23
HyperPlonk accumulates share grid 1703936) are reported apart."""
import glob
import os
import sqlite3
import sys

# bench.py LEG_TAGS, inverted (kept in one place there; copied here so the
# script runs without importing the bench)
LEGS = {1: "msm_2p24", 2: "sumcheck", 3: "msm_host", 4: "scaling", 5: "mle_open", 6: "logup",
        7: "hyperplonk", 8: "msm_2p20", 9: "cpu_baseline", 10: "probe_msm", 11: "probe_sumcheck",
        12: "probe_logup", 13: "probe_mle", 14: "probe_cal", 15: "msm_oneshot",
        16: "zerocheck"}
MARKER = "k_trace_marker"


def _short(name):
    return name.split("(")[0].replace("void ", "")[:60]


def rows_by_leg(db):
    """[(leg, name, grid_x, wg_x, duration_ns, vgpr, scratch, lds)] in dispatch order"""
    c = sqlite3.connect(db)
    cur = c.execute("select pid, name, grid_x, workgroup_x, start, duration, vgpr_count, "
                    "scratch_size, lds_size from kernels order by pid, start")
    out, leg, last_pid = [], "pre", None
    for pid, name, gx, wx, _start, dur, vg, scr, lds in cur:
        if pid != last_pid:
            leg, last_pid = "pre", pid
        if MARKER in name:
            tag = gx // max(wx, 1)
            leg = LEGS.get(tag, f"tag{tag}")
            continue
        out.append((leg, name, gx, wx, dur, vg, scr, lds))
    return out


def summarize(rows, sub="", by_leg=True):
    agg = {}
    for leg, name, gx, wx, dur, vg, scr, lds in rows:
        if sub and sub not in name:
            continue
        key = (leg if by_leg else "", _short(name), gx, wx)
        a = agg.setdefault(key, [0, 0.0, 0, 0, 0])
        a[0] += 1
        a[1] += dur
        a[2], a[3], a[4] = max(a[2], vg), max(a[3], scr), max(a[4], lds)
    return sorted(agg.items(), key=lambda kv: -kv[1][1])


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    by_leg = "--legs" in sys.argv
    p = args[0]
    f = p if p.endswith(".db") else glob.glob(os.path.join(p, "**", "*.db"), recursive=True)[0]
    sub = args[1] if len(args) > 1 else ""
    rows = rows_by_leg(f)
    lw = 13 if by_leg else 0
    print((f"{'leg':{lw}s} " if by_leg else "") +
          f"{'kernel':60s} {'grid':>9s} {'wg':>5s} {'n':>5s} {'avg_us':>9s} {'tot_us':>10s} "
          f"{'vgpr':>5s} {'scr':>5s} {'lds':>6s}")
    for (leg, short, gx, wx), (n, tot, vg, scr, lds) in summarize(rows, sub, by_leg):
        print((f"{leg:{lw}s} " if by_leg else "") +
              f"{short:60s} {gx:9d} {wx:5d} {n:5d} {tot / n / 1e3:9.2f} {tot / 1e3:10.1f} "
              f"{vg:5d} {scr:5d} {lds:6d}")


if __name__ == "__main__":
    main()
