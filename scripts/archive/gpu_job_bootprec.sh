#!/bin/bash
# bootstrap precision sweep (EvalMod parameters) + the KWaySort235 size table
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out
for a in "16 4096 5 5 512 6 88 11" "16 4096 5 5 512 6 88 10" "16 4096 5 5 512 6 88 12" "16 4096 5 5 512 6 119 11" "16 4096 5 5 512 7 88 11" "16 4096 5 5 1024 7 88 11" "16 4096 3 3 512 6 88 11" "16 256 5 5 512 6 88 11"; do
  timeout -k 10 300 python -u scripts/boot_precision.py $a >> gpurun_out/bootprec.jsonl 2>>gpurun_out/bootprec.err || { echo "fail $a"; tail -5 gpurun_out/bootprec.err; exit 1; }
  tail -1 gpurun_out/bootprec.jsonl
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_bootstrap.py -x -v --timeout 600 --timeout-method thread -k kway235 > gpurun_out/kway235.log 2>&1 || { echo "kway235 failed"; tail -30 gpurun_out/kway235.log; exit 1; }
tail -3 gpurun_out/kway235.log
