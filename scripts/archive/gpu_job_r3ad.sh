#!/bin/bash
# MEHP24 kernel trace (kept in full) for a launch-size analysis
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3ad
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d "$R/$O/trace" -o run -- python3 "$R/bench.py" --workload mehp24 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
gzip -f $O/trace/run_kernel_trace.csv
echo ALLOK
