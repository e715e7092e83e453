#!/bin/bash
# SQ issue/stall counters of the NTT passes over one N=1024 sort (one lane)
# usage: gpu_job_sqpmc.sh TAG [regex]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
TAG=${1:-sq}; RX=${2:-k_ntt}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -s KILL 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES --kernel-include-regex "$RX" --output-format csv -d "$R/$O/pmc" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --lanes 1 > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
python - "$O/pmc/run_counter_collection.csv" <<'PY' | tee $O/sq_summary.txt
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r['Kernel_Name']
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    if r['Counter_Name'] == 'SQ_WAVES':
        n[k] += 1
for k, c in sorted(acc.items(), key=lambda kv: -kv[1]['SQ_WAVE_CYCLES']):
    wc = c['SQ_WAVE_CYCLES'] or 1
    print(f"{k[:60]:60s} launches={n[k]:5d} waves/l={c['SQ_WAVES']/max(n[k],1):8.0f} "
          f"wait={c['SQ_WAIT_ANY']/wc:.2f} issue_stall={c['SQ_WAIT_INST_ANY']/wc:.2f} active={c['SQ_ACTIVE_INST_ANY']/wc:.2f} "
          f"valu_active={c['SQ_ACTIVE_INST_VALU']/wc:.2f} valu_insts/wave={c['SQ_INSTS_VALU']/max(c['SQ_WAVES'],1):.0f} "
          f"vmem_rd/wave={c['SQ_INSTS_VMEM_RD']/max(c['SQ_WAVES'],1):.0f}")
PY
gzip -f $O/pmc/run_counter_collection.csv
echo ALLOK
