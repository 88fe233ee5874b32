"""Summarise a rocprofv3 SQLite trace (kernel-trace) into profiles/: the
per-kernel statistics table (csv + txt) and the headline kernels' per-launch
durations, grouped by grid size (one group per MSM size)."""
import sqlite3, sys, collections, csv
db, out_prefix, title = sys.argv[1], sys.argv[2], sys.argv[3]
c = sqlite3.connect(db)
rows = list(c.execute('select name, duration, grid_x, workgroup_x, vgpr_count, lds_size from kernels order by start'))
agg = collections.OrderedDict()
for name, dur, gx, wx, vg, lds in rows:
    a = agg.setdefault(name, [0, 0.0, vg, lds])
    a[0] += 1; a[1] += dur
tot = sum(a[1] for a in agg.values())
with open(out_prefix + '_kernel_stats.csv', 'w', newline='') as f:
    w = csv.writer(f); w.writerow(['kernel', 'calls', 'total_ms', 'avg_us', 'pct', 'vgpr', 'lds'])
    for n, (k, s, vg, lds) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        w.writerow([n, k, round(s / 1e6, 3), round(s / k / 1e3, 2), round(100 * s / tot, 2), vg, lds])
with open(out_prefix + '_kernel_stats_summary.txt', 'w') as f:
    f.write(title + '\n')
    f.write('%-60s %7s %11s %11s %6s\n' % ('kernel', 'calls', 'total_ms', 'avg_us', 'pct'))
    for n, (k, s, vg, lds) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        f.write('%-60s %7d %11.3f %11.2f %6.2f\n' % (n[:60], k, s / 1e6, s / k / 1e3, 100 * s / tot))
    f.write('\nheadline kernels by launch grid (grid_x = work-items; one group per problem size)\n')
    for key in ('k_msm_accumulate', 'k_logup(', 'k_sc_round', 'k_sc_persist'):
        groups = collections.OrderedDict()
        for name, dur, gx, wx, vg, lds in rows:
            if key in name:
                groups.setdefault((name.split('(')[0], gx), []).append(dur)
        for (n, gx), ds in groups.items():
            f.write('  %-28s grid_x=%-10d launches=%-4d avg_us=%10.2f min_us=%10.2f\n' % (n, gx, len(ds), sum(ds) / len(ds) / 1e3, min(ds) / 1e3))
    acc = [dur for name, dur, *_ in rows if 'k_msm_accumulate' in name]
    f.write('\nheadline MSM (bench.py: 2 warmup + 5 timed 2^24 commitments = the first 7 '
            'k_msm_accumulate launches): ' + ', '.join('%.2f' % (d / 1e6) for d in acc[:7]) +
            ' ms; timed avg %.3f ms\n' % (sum(acc[2:7]) / 5 / 1e6))
print(open(out_prefix + '_kernel_stats_summary.txt').read())
