#!/usr/bin/env python3
"""Compiler resource usage (VGPR/AGPR, spills, waves per SIMD, LDS) of the
kernels of one gfx950 source, filtered by a regex on the demangled name.
usage: res_usage.py SOURCE [regex] [extra hipcc flags...]"""
import re
import subprocess
import sys

src = sys.argv[1]
rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else '.')
out = subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-ffp-contract=off',
                      '-Wno-unused-function', '-Rpass-analysis=kernel-resource-usage', '-c', src, '-o', '/dev/null']
                     + sys.argv[3:], capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        dem = subprocess.run(['c++filt', m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = {'name': re.sub(r'\(.*', '', dem.replace('(anonymous namespace)::', '').replace('void fhe::dev::', ''))}
        rows.append(cur)
        continue
    m = re.search(r'remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)', line)
    if m and cur is not None:
        cur[m.group(1).strip()] = int(m.group(2))
for r in rows:
    if rx.search(r['name']):
        print(f"{r['name']:60s} vgpr {r.get('VGPRs', 0):4d} agpr {r.get('AGPRs', 0):3d} spill {r.get('VGPRs Spill', 0):3d} "
              f"waves/SIMD {r.get('Occupancy', 0)} lds {r.get('LDS Size', 0)}")
