"""Summarise a rocprofv3 kernel-trace CSV: time share per kernel and the
achieved HBM bandwidth of the NTT passes (algorithmic bytes: every limb is
read and written once per pass)."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
stat = collections.defaultdict(list)
for r in rows:
    m = re.search(r'(k_[a-z0-9_]+(<[^>]*>)?)\(', r['Kernel_Name'])
    name = m.group(1) if m else r['Kernel_Name'][:40]
    dur = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    stat[name].append((dur, int(r['Grid_Size_X']), int(r['Grid_Size_Y']), int(r['Grid_Size_Z']), r['VGPR_Count'],
                       r['LDS_Block_Size']))
tot_all = sum(x[0] for v in stat.values() for x in v)
print(f'total kernel time {tot_all / 1e6:.2f} ms over {len(rows)} dispatches')
for k, v in sorted(stat.items(), key=lambda kv: -sum(x[0] for x in kv[1]))[:16]:
    tot = sum(x[0] for x in v)
    print(f'{k:34s} n={len(v):6d} {tot / 1e6:9.2f} ms {100 * tot / tot_all:5.1f}%  avg {tot / len(v) / 1e3:7.2f} us'
          f'  vgpr={v[0][4]} lds={v[0][5]}')
# NTT passes launch grid (segments x 256 threads, blocks per limb, limbs)
for k in sorted(stat):
    if not k.startswith('k_ntt'):
        continue
    v = stat[k]
    limbs = [gx // 256 * gz for _, gx, _, gz, _, _ in v]
    tb = sum(L * n * 16 for L in limbs)
    tt = sum(x[0] for x in v)
    print(f'{k}: {tb / tt:.1f} GB/s algorithmic (one read + one write per coefficient), '
          f'avg {sum(limbs) / len(v):.1f} limbs/launch, avg {tt / len(v) / 1e3:.2f} us')
