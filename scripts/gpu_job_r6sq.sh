#!/bin/bash
# round 6: SQ issue / stall counters of the ModDown + rescale conversion, fp64 and
# 128-bit forms, over 32 members at ell = 40 and 24 (scripts/conv_micro.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_sq}
mkdir -p $O
export TMPDIR=/tmp
for fp in 0 1; do
  FHE_MODDOWN_FP=$fp timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM --kernel-include-regex "k_moddown" --output-format csv -d "$R/$O/pmc$fp" -o run -- python3 "$R/scripts/conv_micro.py" moddown_rescale32 40,24 > $O/pmc$fp.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc$fp.log; exit 1; }
done
for fp in 0 1; do
python - "$O/pmc$fp/run_counter_collection.csv" <<'PY' | tee -a $O/sq_summary.txt
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = r['Kernel_Name'][:70] + ' grid=' + r.get('Grid_Size', '?')
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, c in acc.items():
    wc = c['SQ_WAVE_CYCLES'] or 1
    print(f"{k:90s} wait={c['SQ_WAIT_ANY']/wc:.2f} issue_stall={c['SQ_WAIT_INST_ANY']/wc:.2f} active={c['SQ_ACTIVE_INST_ANY']/wc:.2f} "
          f"valu_active={c['SQ_ACTIVE_INST_VALU']/wc:.2f} valu={c['SQ_INSTS_VALU']:.3g} lds={c['SQ_INSTS_LDS']:.3g} smem={c['SQ_INSTS_SMEM']:.3g} wave_cycles={wc:.3g}")
PY
done
gzip -f $O/pmc*/run_counter_collection.csv
