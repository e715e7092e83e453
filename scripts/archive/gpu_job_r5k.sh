#!/bin/bash
# round 5: FP row epilogue operands loaded late (ab_epi0) -- parity, bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_k}
mkdir -p $O
FHE_LIB=fhe-sorting_amd/lib/ab_epi0.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_base.json 2> $O/bench_base.err && \
FHE_LIB=fhe-sorting_amd/lib/ab_epi0.so timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_epi0.json 2> $O/bench_epi0.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_base2.json 2> $O/bench_base2.err && \
FHE_LIB=fhe-sorting_amd/lib/ab_epi0.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_epi02.json 2> $O/bench_epi02.err
