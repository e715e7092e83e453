#!/bin/bash
# round 3: the full GPU suite (parity, digests, wire, collectives, k-way, MEHP24)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -5 $O/gpu_tests.log
grep -E "FAILED|Error" $O/gpu_tests.log | head -20
exit $rc
