#!/bin/bash
# round 5: leaf sums with byte-aligned window extracts and the two-term Shoup
# epilogue -- MFMA/digest parity, A/B vs the committed kernels.hip (lib/ab_leafold.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_n}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_digests.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
FHE_LIB=fhe-sorting_amd/lib/ab_leafold.so timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_old.json 2> $O/bench_old.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_new.json 2> $O/bench_new.err && \
FHE_LIB=fhe-sorting_amd/lib/ab_leafold.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_old2.json 2> $O/bench_old2.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_new2.json 2> $O/bench_new2.err
