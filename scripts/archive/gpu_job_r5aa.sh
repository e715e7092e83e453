#!/bin/bash
# round 5: ModUp fold with the next wave-step's sources prefetched
# (lib/ab_pf.so, -DFHE_MUF_PREFETCH=1) -- parity of the forced fold, A/B of the
# ModUp family on the N=1024 sort (fold forced) and MEHP24
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_aa}
mkdir -p $O
FHE_LIB=fhe-sorting_amd/lib/ab_pf.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fold_env.py tests/test_gpu_mfma.py tests/test_gpu_mehp24.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_def.json 2> $O/bench_def.err && \
FHE_MODUP_FOLD=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_fold.json 2> $O/bench_fold.err && \
FHE_MODUP_FOLD=1 FHE_LIB=fhe-sorting_amd/lib/ab_pf.so timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_pf.json 2> $O/bench_pf.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 > $O/mehp_def.json 2> $O/mehp_def.err && \
FHE_LIB=fhe-sorting_amd/lib/ab_pf.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 > $O/mehp_pf.json 2> $O/mehp_pf.err
