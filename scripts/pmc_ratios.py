"""Summarise SQ counters per kernel (and grid size) from a rocprofv3 --pmc CSV:
wave-cycle breakdown (parked on waitcnt / issue-stalled / active) and VALU
instructions per wave."""
import collections
import csv
import sys

rows = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    name = r['Kernel_Name'].split('(')[0].replace('void fhe::dev::(anonymous namespace)::', '')
    key = (name, int(r['Grid_Size']), int(r['VGPR_Count']))
    rows[key][r['Counter_Name']].append(float(r['Counter_Value']))
for (name, grid, vgpr), c in sorted(rows.items()):
    m = {k: sum(v) / len(v) for k, v in c.items()}
    wc = m.get('SQ_WAVE_CYCLES', 0) or 1
    waves = m.get('SQ_WAVES', 0) or 1
    print(f"{name:40s} grid {grid:9d} vgpr {vgpr:3d} n={len(c['SQ_WAVES'])} "
          f"waitany {m.get('SQ_WAIT_ANY', 0) / wc:.2f} waitinst {m.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} "
          f"active {m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} valu/act {m.get('SQ_ACTIVE_INST_VALU', 0) / max(1, m.get('SQ_ACTIVE_INST_ANY', 1)):.2f} "
          f"valu_insts/wave {m.get('SQ_INSTS_VALU', 0) / waves:.0f} wavecyc/wave {wc / waves:.0f} busy {m.get('SQ_BUSY_CYCLES', 0):.0f}")
