"""Fold rocprofv3 --pmc CSVs (one FETCH_SIZE pass, one WRITE_SIZE pass, each
--output-format csv) into per-kernel HBM bytes per launch.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE/WRITE_SIZE are in
KiB; FETCH_SIZE reports half the bytes of a wide streaming read, so it is
doubled.  The NTT moves 8 B per lane (an uncalibrated width), so the figure is
the guide's correction applied as-is.
usage: pmc_summary.py fetch_counter_collection.csv write_counter_collection.csv out.json
"""
import collections
import csv
import json
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from pmc_meta import meta, region  # noqa: E402


def load(path, counter):
    acc = collections.defaultdict(lambda: [0, 0.0])
    rows, found = region(list(csv.DictReader(open(path))))
    print(f'{path}: {"region markers found" if found else "no region markers: every dispatch"}', file=sys.stderr)
    for r in rows:
        if r['Counter_Name'] != counter:
            continue
        m = re.search(r'(k_[a-z0-9_]+(<[^>]*>)?)\(', r['Kernel_Name'])
        name = m.group(1) if m else r['Kernel_Name'][:40]
        a = acc[name]
        a[0] += 1
        a[1] += float(r['Counter_Value'])
    return acc


f = load(sys.argv[1], 'FETCH_SIZE')
w = load(sys.argv[2], 'WRITE_SIZE')
out = {}
for k in sorted(set(f) & set(w)):
    fk = f[k][1] / f[k][0]
    wk = w[k][1] / w[k][0]
    out[k] = {'launches': f[k][0], 'fetch_size_kib': round(fk, 1), 'write_size_kib': round(wk, 1),
              'hbm_bytes_per_launch': round((2 * fk + wk) * 1024)}
for k, v in out.items():
    print(k, v)
out['_meta'] = meta()
json.dump(out, open(sys.argv[3], 'w'), indent=1)
