#!/bin/bash
# round 3, first call: OpenFHE PS split -- parity vs oracle, the 40-bit
# reference context at N = 256/512/1024, precision diag for both splits
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out/r3a
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "chebyshev or doubled_sinc or direct_sort_bit_exact or multi_batch or batched_ops" > gpurun_out/r3a/parity.log 2>&1 \
  || { echo "parity failed"; tail -40 gpurun_out/r3a/parity.log; exit 1; }
tail -3 gpurun_out/r3a/parity.log
timeout -k 10 900 python -u scripts/diag_precision.py 1024:40:16:1 256:40:17:1 512:40:17:1 1024:40:17:1 1024:40:16:0 > gpurun_out/r3a/diag.jsonl 2> gpurun_out/r3a/diag.err \
  || { echo "diag failed"; tail -20 gpurun_out/r3a/diag.err; exit 1; }
cat gpurun_out/r3a/diag.jsonl
echo ALLOK
