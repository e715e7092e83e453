#!/bin/bash
# round 5: fp64 epilogue of the folded MFMA sums for primes < 2^41 (leaf sums,
# ModUp, ModDown+rescale) -- parity with every fold on, A/B against the
# closing-profile library (lib/ab_base.so) on the N=1024 sort and MEHP24
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_u}
mkdir -p $O
FHE_MODDOWN_FOLD=1 FHE_MODUP_FOLD=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_mehp24.py tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
FHE_LIB=fhe-sorting_amd/lib/ab_base.so timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_base.json 2> $O/bench_base.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_00.json 2> $O/bench_00.err && \
FHE_MODDOWN_FOLD=1 FHE_MODUP_FOLD=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_11.json 2> $O/bench_11.err && \
FHE_MODDOWN_FOLD=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_10.json 2> $O/bench_10.err && \
FHE_LIB=fhe-sorting_amd/lib/ab_base.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_baseb.json 2> $O/bench_baseb.err && \
FHE_MODDOWN_FOLD=1 FHE_MODUP_FOLD=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_11b.json 2> $O/bench_11b.err && \
FHE_LIB=fhe-sorting_amd/lib/ab_base.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 > $O/mehp_base.json 2> $O/mehp_base.err && \
FHE_MODDOWN_FOLD=1 FHE_MODUP_FOLD=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 > $O/mehp_11.json 2> $O/mehp_11.err
