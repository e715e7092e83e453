#!/bin/bash
# kernel trace of 6 bootstraps (config 4 context)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/boot_prof.py > $O/plain.log 2>&1 || { echo "plain failed"; tail -5 $O/plain.log; exit 1; }
cat $O/plain.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o run -- python3 "$R/scripts/boot_prof.py" > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
python scripts/trace_summary.py $O/trace/run_kernel_trace.csv > $O/trace_summary.txt && head -40 $O/trace_summary.txt
gzip -f $O/trace/run_kernel_trace.csv
echo ALLOK
