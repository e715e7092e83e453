#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3n
mkdir -p $O
timeout -k 10 300 python3 scripts/batch_probe.py > $O/batch_probe.log 2>&1 || { echo "probe failed"; tail -5 $O/batch_probe.log; exit 1; }
cat $O/batch_probe.log
echo ALLOK
