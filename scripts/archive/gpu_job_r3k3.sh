#!/bin/bash
# k-way (config 4): kernel trace (dispatch count), then the PMC passes for its
# dominant kernels with the 131072-packet AQL ring (the profiler's ring-wrap
# bug), then the bench line reading the tables
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3k3
mkdir -p $O
export TMPDIR=/tmp FHE_FAULT_REPORT=1 ROC_AQL_QUEUE_SIZE=131072
(while sleep 50; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
B="--workload kway --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --lanes 1"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o run -- python3 "$R/bench.py" $B > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
python scripts/trace_summary.py $O/trace/run_kernel_trace.csv > $O/trace_summary.txt && head -20 $O/trace_summary.txt
gzip -f $O/trace/run_kernel_trace.csv
RX='k_lt_inner|k_ntt_fwd<8, 4, true|k_ntt_inv|k_modup_convert|k_ks_inner|k_tensor'
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 420 rocprofv3 --pmc $C --kernel-include-regex "$RX" --output-format csv -d "$R/$O/pmc_$C" -o run -- python3 "$R/bench.py" $B > $O/pmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"
  [ $rc -eq 0 ] || { grep -A8 "fhe fault report\] SIG" $O/pmc_$C.log | head -20; tail -5 $O/pmc_$C.log; exit 1; }
done
timeout -s KILL 420 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$RX" --output-format csv -d "$R/$O/pmc_SQ" -o run -- python3 "$R/bench.py" $B > $O/pmc_SQ.log 2>&1 || { echo "pmc SQ failed"; tail -5 $O/pmc_SQ.log; exit 1; }
python scripts/pmc_summary.py $O/pmc_FETCH_SIZE/run_counter_collection.csv $O/pmc_WRITE_SIZE/run_counter_collection.csv $O/pmc_traffic_kway.json > $O/pmc_traffic_kway.txt || exit 1
python scripts/pmc_sq_summary.py $O/pmc_SQ/run_counter_collection.csv $O/pmc_sq_kway.json > $O/pmc_sq_kway.txt || exit 1
gzip -f $O/pmc_*/run_counter_collection.csv
cp $O/pmc_traffic_kway.json $O/pmc_sq_kway.json profiles/
timeout -k 10 500 python bench.py --workload kway --steps 2 --no-cpu-baseline > $O/bench_kway.json 2> $O/bench_kway.err || { echo "bench failed"; tail -5 $O/bench_kway.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_kway.json'));r=d['roofline'];print(d['ms_per_step'], r['kernel'], r['frac'], r.get('traffic'), r.get('valu_frac'), r.get('run_op'))"
echo ALLOK
