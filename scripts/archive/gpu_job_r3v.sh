#!/bin/bash
# kernel trace of 6 bootstraps after double hoisting + stage split
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/boot_stages.py 16 4096 > $O/boot_stages.json 2> $O/boot_stages.err || { echo "stages failed"; tail -5 $O/boot_stages.err; exit 1; }
cat $O/boot_stages.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o run -- python3 "$R/scripts/boot_prof.py" > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
gzip -f $O/trace/run_kernel_trace.csv
echo ALLOK
