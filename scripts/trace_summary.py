"""Summarise a rocprofv3 kernel-trace CSV: time share per kernel.

When the run carries region markers (bench.py FHE_PROF_REGION=1: k_region_begin
/ k_region_end around the timed sort), only the dispatches inside the region are
counted, and `--stats-out PATH` writes them in rocprofv3's --stats layout
(Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev):
profiles/r4_*/region_kernel_stats.csv, from which bench.py's roofline line can
be recomputed (its live clock runs the same one-lane sort).
usage: trace_summary.py run_kernel_trace.csv [--stats-out PATH]
"""
import collections
import csv
import math
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_meta import region  # noqa: E402

args = [a for a in sys.argv[1:]]
stats_out = None
if '--stats-out' in args:
    i = args.index('--stats-out')
    stats_out = args[i + 1]
    del args[i:i + 2]
rows, found = region(list(csv.DictReader(open(args[0]))))
print(f'region: {"k_region_begin..k_region_end" if found else "none (every dispatch)"}')
stat = collections.defaultdict(list)
full = {}
for r in rows:
    if 'k_region_' in r['Kernel_Name']:
        continue
    m = re.search(r'(k_[a-z0-9_]+(<[^>]*>)?)\(', r['Kernel_Name'])
    name = m.group(1) if m else r['Kernel_Name'][:40]
    full[name] = r['Kernel_Name']
    dur = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    stat[name].append((dur, int(r['Grid_Size_X']), int(r['Grid_Size_Y']), int(r['Grid_Size_Z']), r['VGPR_Count'],
                       r['LDS_Block_Size'], r.get('Accum_VGPR_Count', ''), r.get('SGPR_Count', '')))
tot_all = sum(x[0] for v in stat.values() for x in v)
print(f'total kernel time {tot_all / 1e6:.2f} ms over {sum(len(v) for v in stat.values())} dispatches')
for k, v in sorted(stat.items(), key=lambda kv: -sum(x[0] for x in kv[1]))[:24]:
    tot = sum(x[0] for x in v)
    print(f'{k:34s} n={len(v):6d} {tot / 1e6:9.2f} ms {100 * tot / tot_all:5.1f}%  avg {tot / len(v) / 1e3:7.2f} us'
          f'  vgpr={v[0][4]} agpr={v[0][6]} sgpr={v[0][7]} lds={v[0][5]}')
# (algorithmic bytes per launch come from the engine's own launch wrappers --
# bench.py's live clock, `roofline.kernels` -- not from grid shapes here: the
# register-only row passes and the column passes lay their grids out differently)
if stats_out:
    with open(stats_out, 'w', newline='') as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'Percentage', 'MinNs', 'MaxNs', 'StdDev'])
        for k, v in sorted(stat.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
            d = [x[0] for x in v]
            tot = sum(d)
            avg = tot / len(d)
            sd = math.sqrt(sum((x - avg) ** 2 for x in d) / len(d))
            w.writerow([full[k], len(d), tot, round(avg, 6), round(100 * tot / tot_all, 2), min(d), max(d), round(sd, 6)])
