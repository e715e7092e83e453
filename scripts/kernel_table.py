#!/usr/bin/env python3
"""DESIGN.md §5 counter table of one profiled build: for every NTT pass (and the
other kernels above a time share), from a profiles/r4_* directory --
  share of the sort and average duration (region_kernel_stats.csv, the sort
  alone), HBM fraction (algorithmic bytes from the bench line's live clock /
  the trace's duration), PMC traffic / algorithmic bytes (pmc_traffic.json),
  VALU fraction (pmc_sq.json x valu_mix.json, as bench.py), the wave-cycle split
  (waitcnt / issue stall, SQ_WAIT_ANY / SQ_WAIT_INST_ANY over SQ_WAVE_CYCLES),
  and the registers and waves per SIMD the compiler gives the instantiation
  (-Rpass-analysis=kernel-resource-usage of the sources that built it).
usage: kernel_table.py PROFILE_DIR [min_share]
"""
import csv
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
d = sys.argv[1]
min_share = float(sys.argv[2]) if len(sys.argv) > 2 else 0.01


def short(name):
    m = re.search(r'(k_[a-z0-9_]+(<[^>]*>)?)\(', name)
    return m.group(1) if m else name


stats = {}
for r in csv.DictReader(open(os.path.join(d, 'region_kernel_stats.csv'))):
    stats[short(r['Name'])] = (int(r['Calls']), float(r['TotalDurationNs']), float(r['AverageNs']))
total = sum(v[1] for v in stats.values())
bench = json.load(open(os.path.join(d, 'bench.json')))
clock = bench['roofline']['kernels']  # by symbol: avg_us, GBps, launches (top entries)
traffic = json.load(open(os.path.join(d, 'pmc_traffic.json')))
sq = json.load(open(os.path.join(d, 'pmc_sq.json')))
mix = json.load(open(os.path.join(REPO, 'profiles', 'valu_mix.json')))

# compiler resources: VGPRs (+AGPRs), waves per SIMD, LDS per block
res = {}
for src in ('ntt.hip', 'kernels.hip'):
    out = subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-ffp-contract=off',
                          '-Wno-unused-function', '-Rpass-analysis=kernel-resource-usage', '-c',
                          os.path.join(REPO, 'fhe-sorting_amd', 'csrc', 'device', src), '-o', '/dev/null'],
                         capture_output=True, text=True).stderr
    cur = None
    for line in out.splitlines():
        m = re.search(r'Function Name: (\S+)', line)
        if m:
            dem = subprocess.run(['c++filt', m.group(1)], capture_output=True, text=True).stdout.strip()
            cur = short(dem + '(')
            res[cur] = {}
            continue
        m = re.search(r'remark:\s+(VGPRs|AGPRs|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)', line)
        if m and cur:
            res[cur][m.group(1).split(' ')[0]] = int(m.group(2))

print('| kernel | share | avg µs | HBM frac | PMC / alg. | VALU frac | waitcnt | issue stall | VGPR (+AGPR) | waves/SIMD | LDS KB |')
print('|---|---|---|---|---|---|---|---|---|---|---|')
for k, (calls, tot, avg) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
    share = tot / total
    if share < min_share:
        continue
    c = clock.get(k)
    frac = f'{c["GBps"] / 8000:.2f}' if c else ''
    alg = c and c['GBps'] * 1e9 * c['avg_us'] * 1e-6
    t = traffic.get(k)
    ratio = f'{t["hbm_bytes_per_launch"] / alg:.2f}' if (t and alg) else ''
    s = sq.get(k)
    vf = wait = stall = ''
    if s and k in mix and 'SQ_INSTS_VALU' in s:
        vs = s['SQ_INSTS_VALU'] * 64 * mix[k]['ps_per_lane_instr'] * 1e-12
        vf = f'{vs / (avg * 1e-9):.2f}'
        wc = s.get('SQ_WAVE_CYCLES') or 1
        wait = f'{s.get("SQ_WAIT_ANY", 0) / wc:.2f}'
        stall = f'{s.get("SQ_WAIT_INST_ANY", 0) / wc:.2f}'
    r = res.get(k, {})
    vg = f'{r.get("VGPRs", "")}' + (f' (+{r["AGPRs"]})' if r.get('AGPRs') else '')
    print(f'| `{k}` | {100 * share:.1f}% | {avg / 1e3:.1f} | {frac} | {ratio} | {vf} | {wait} | {stall} | {vg} | '
          f'{r.get("Occupancy", "")} | {r.get("LDS", 0) / 1024:.1f} |')
