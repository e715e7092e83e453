#!/bin/bash
# bootstrapping: GPU parity tests, then k-way-with-bootstrap runs (k M logN d_g ...)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bootstrap.py -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_boot.log 2>&1 || { echo "boot tests failed"; tail -40 gpurun_out/tests_boot.log; exit 1; }
tail -12 gpurun_out/tests_boot.log
while [ $# -ge 4 ]; do
  timeout -k 10 900 python -u scripts/kway_boot_run.py $1 $2 $3 $4 >> gpurun_out/kway_boot.jsonl 2>gpurun_out/kway_boot.err || { echo "kway run $1 $2 failed"; tail -20 gpurun_out/kway_boot.err; exit 1; }
  tail -1 gpurun_out/kway_boot.jsonl
  shift 4
done
echo ALLOK
