"""Per-kernel summary (launch shape, count, average/total us, VGPRs, scratch)
of a rocprofv3 SQLite output (ROCm 7 rocpd format):
python profiles/kstats.py <dir-or-db> [name-substring]"""
import glob
import os
import sqlite3
import sys


def main():
    p = sys.argv[1]
    f = p if p.endswith(".db") else glob.glob(os.path.join(p, "**", "*.db"), recursive=True)[0]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    c = sqlite3.connect(f)
    rows = c.execute("select name, grid_x, workgroup_x, count(*), avg(duration), sum(duration), "
                     "max(vgpr_count), max(scratch_size), max(lds_size) from kernels "
                     "group by name, grid_x, workgroup_x order by sum(duration) desc")
    print(f"{'kernel':60s} {'grid':>9s} {'wg':>5s} {'n':>5s} {'avg_us':>9s} {'tot_us':>10s} "
          f"{'vgpr':>5s} {'scr':>5s} {'lds':>6s}")
    for name, gx, wx, n, avg, tot, vg, scr, lds in rows:
        short = name.split("(")[0].replace("void ", "")[:60]
        if sub and sub not in name:
            continue
        print(f"{short:60s} {gx:9d} {wx:5d} {n:5d} {avg / 1e3:9.2f} {tot / 1e3:10.1f} "
              f"{vg:5d} {scr:5d} {lds:6d}")


if __name__ == "__main__":
    main()
