#!/bin/bash
# round 5: fp64 NTT for the 40-bit limbs -- NTT / parity tests, then the full
# GPU suite, then the bench A/B (FHE_NTT_FP=0 integer-only vs default)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_a}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1 && \
FHE_NTT_FP=0 timeout -k 10 300 python bench.py > $O/bench_fp0.json 2> $O/bench_fp0.err && \
timeout -k 10 300 python bench.py > $O/bench_fp1.json 2> $O/bench_fp1.err
