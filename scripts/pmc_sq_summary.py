"""Fold one rocprofv3 --pmc pass of SQ counters into per-kernel per-launch
averages (profiles/pmc_sq*.json, read by bench.py for roofline.valu_frac).

Kernel names are normalised like scripts/pmc_summary.py (the instantiation,
e.g. 'k_linear_sum_multi<10>').  SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* / SQ_WAIT_*
count quad-cycles on gfx950 (MI355X_MICROARCH.md, PMC units table).
usage: pmc_sq_summary.py counter_collection.csv out.json
"""
import collections
import csv
import json
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from pmc_meta import meta, region  # noqa: E402

acc = collections.defaultdict(lambda: collections.defaultdict(float))
launches = collections.defaultdict(set)
rows, found = region(list(csv.DictReader(open(sys.argv[1]))))
print(f'{sys.argv[1]}: {"region markers found" if found else "no region markers: every dispatch"}', file=sys.stderr)
for r in rows:
    m = re.search(r'(k_[a-z0-9_]+(<[^>]*>)?)\(', r['Kernel_Name'])
    name = m.group(1) if m else r['Kernel_Name'][:40]
    acc[name][r['Counter_Name']] += float(r['Counter_Value'])
    launches[name].add(r.get('Dispatch_Id') or r.get('Correlation_Id') or len(launches[name]))
out = {}
for k, c in sorted(acc.items()):
    n = max(1, len(launches[k]))
    out[k] = {'launches': n, **{cn: round(v / n, 1) for cn, v in sorted(c.items())}}
for k, v in out.items():
    w = v.get('SQ_WAVE_CYCLES', 0) or 1
    print(f"{k:45s} n={v['launches']:5d} waves={v.get('SQ_WAVES', 0):9.0f} valu_insts/wave="
          f"{v.get('SQ_INSTS_VALU', 0) / max(1, v.get('SQ_WAVES', 1)):7.0f} valu_active/wavecyc="
          f"{v.get('SQ_ACTIVE_INST_VALU', 0) / w:.2f} wait={v.get('SQ_WAIT_ANY', 0) / w:.2f} "
          f"issue_stall={v.get('SQ_WAIT_INST_ANY', 0) / w:.2f}")
out['_meta'] = meta()
json.dump(out, open(sys.argv[2], 'w'), indent=1)
