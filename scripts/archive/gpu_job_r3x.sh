#!/bin/bash
# DirectSort kernel trace on the current build (one lane, one sort)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o run -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --lanes 1 > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
python scripts/trace_summary.py $O/trace/run_kernel_trace.csv > $O/trace_summary.txt && head -36 $O/trace_summary.txt
gzip -f $O/trace/run_kernel_trace.csv
echo ALLOK
