#!/bin/bash
# k-way GPU tests (network parity, SortUtils known answers, bootstrapping) + config-4 runs
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kway.py tests/test_gpu_bootstrap.py tests/test_gpu_reference_suites.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_kway.log 2>&1 || { echo "kway tests failed"; tail -40 gpurun_out/tests_kway.log; exit 1; }
tail -3 gpurun_out/tests_kway.log
while [ $# -ge 4 ]; do
  timeout -k 10 900 python -u scripts/kway_boot_run.py $1 $2 $3 $4 >> gpurun_out/kway_boot.jsonl 2>gpurun_out/kway_boot.err || { echo "kway run $1 $2 failed"; tail -20 gpurun_out/kway_boot.err; exit 1; }
  tail -1 gpurun_out/kway_boot.jsonl
  shift 4
done
echo ALLOK
