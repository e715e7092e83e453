#!/bin/bash
# SQ counters of the MFMA sums-of-products kernels against their VALU forms
# (one lane, one sort; FHE_MFMA=7 then 0), plus the kernel trace of the MFMA build
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r3mfp}
mkdir -p $O
export TMPDIR=/tmp
(while sleep 50; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
B="--steps 1 --warmup 0 --no-cpu-baseline --no-roofline --lanes 1"
RX='k_linear_sum|k_modup|k_moddown_rescale'
for V in 7 0; do
  FHE_MFMA=$V timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --kernel-include-regex "$RX" --output-format csv -d "$R/$O/pmc$V" -o run -- python3 "$R/bench.py" $B > $O/pmc$V.log 2>&1 || { echo "pmc $V failed"; tail -5 $O/pmc$V.log; exit 1; }
  python scripts/pmc_sq_summary.py $O/pmc$V/run_counter_collection.csv $O/sq$V.json || exit 1
  gzip -f $O/pmc$V/run_counter_collection.csv
done
FHE_MFMA=7 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o run -- python3 "$R/bench.py" $B > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
python scripts/trace_summary.py $O/trace/run_kernel_trace.csv > $O/trace_summary.txt && head -24 $O/trace_summary.txt
gzip -f $O/trace/run_kernel_trace.csv
echo ALLOK
