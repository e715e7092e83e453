#!/bin/bash
# round 5: mul_add's summands folded into the tensor pass (k_tensor_lin,
# FHE_TENSOR_LIN=1 default) -- parity, A/B on the N=1024 sort and MEHP24
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_r}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_mehp24.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
FHE_TENSOR_LIN=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_0.json 2> $O/bench_0.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_1.json 2> $O/bench_1.err && \
FHE_TENSOR_LIN=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_0b.json 2> $O/bench_0b.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_1b.json 2> $O/bench_1b.err && \
FHE_TENSOR_LIN=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 > $O/mehp_0.json 2> $O/mehp_0.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 > $O/mehp_1.json 2> $O/mehp_1.err
