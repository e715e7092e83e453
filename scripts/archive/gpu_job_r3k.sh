#!/bin/bash
# MEHP24 (dnum 3) kernel-time profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o run -- python3 "$R/bench.py" --workload mehp24 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --lanes 1 > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
python scripts/trace_summary.py $O/trace/run_kernel_trace.csv > $O/trace_summary.txt && head -40 $O/trace_summary.txt
rm -f $O/trace/run_kernel_trace.csv
echo ALLOK
