#!/bin/bash
# round 3 profile of the headline workload (40-bit, OpenFHE PS split): kernel
# trace + stats, FETCH_SIZE / WRITE_SIZE / SQ counter passes (one lane, one
# sort each), their per-kernel tables in profiles/, then the bench line that
# reads them (roofline.traffic, roofline.valu_frac)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
TAG=${1:-r3e}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
(while sleep 50; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
B="--steps 1 --warmup 0 --no-cpu-baseline --lanes 1"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o run -- python3 "$R/bench.py" $B > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
python scripts/trace_summary.py $O/trace/run_kernel_trace.csv > $O/trace_summary.txt && head -25 $O/trace_summary.txt || exit 1
gzip -f $O/trace/run_kernel_trace.csv
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 600 rocprofv3 --pmc $C --kernel-include-regex 'k_[a-z]' --output-format csv -d "$R/$O/pmc_$C" -o run -- python3 "$R/bench.py" $B --no-roofline > $O/pmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $O/pmc_$C.log; exit 1; }
done
timeout -s KILL 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --kernel-include-regex 'k_[a-z]' --output-format csv -d "$R/$O/pmc_SQ" -o run -- python3 "$R/bench.py" $B --no-roofline > $O/pmc_SQ.log 2>&1 || { echo "pmc SQ failed"; tail -5 $O/pmc_SQ.log; exit 1; }
python scripts/pmc_summary.py $O/pmc_FETCH_SIZE/run_counter_collection.csv $O/pmc_WRITE_SIZE/run_counter_collection.csv $O/pmc_traffic.json > $O/pmc_traffic.txt || exit 1
python scripts/pmc_sq_summary.py $O/pmc_SQ/run_counter_collection.csv $O/pmc_sq.json > $O/pmc_sq.txt || exit 1
gzip -f $O/pmc_*/run_counter_collection.csv
cp $O/pmc_traffic.json profiles/pmc_traffic.json
cp $O/pmc_sq.json profiles/pmc_sq.json
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print(d['ms_per_step'], d['value'], r['kernel'], r['frac'], r.get('traffic'), r.get('valu_frac'), r.get('valu_issue_frac'), r.get('wave_cycle_split'), d.get('cpu_baseline'))"
echo ALLOK
