#!/bin/bash
# round 5: the folded-constant MFMA ModUp conversion (k_modup_fold,
# FHE_MODUP_FOLD=1) -- parity, A/B on the N=1024 sort and MEHP24
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_s}
mkdir -p $O
export FHE_MODUP_FOLD=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_mehp24.py tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
FHE_MODUP_FOLD=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_0.json 2> $O/bench_0.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_1.json 2> $O/bench_1.err && \
FHE_MODUP_FOLD=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_0b.json 2> $O/bench_0b.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_1b.json 2> $O/bench_1b.err && \
FHE_MODUP_FOLD=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 > $O/mehp_0.json 2> $O/mehp_0.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 > $O/mehp_1.json 2> $O/mehp_1.err
