#!/bin/bash
# round 5: the folded-constant MFMA ModDown+rescale conversion
# (k_moddown_rescale_fold, FHE_MODDOWN_FOLD=1) with and without the ModUp one
# (FHE_MODUP_FOLD) -- parity, A/B on the N=1024 sort and MEHP24
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_t}
mkdir -p $O
FHE_MODDOWN_FOLD=1 FHE_MODUP_FOLD=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_mehp24.py tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_00.json 2> $O/bench_00.err && \
FHE_MODDOWN_FOLD=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_10.json 2> $O/bench_10.err && \
FHE_MODDOWN_FOLD=1 FHE_MODUP_FOLD=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_11.json 2> $O/bench_11.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_00b.json 2> $O/bench_00b.err && \
FHE_MODDOWN_FOLD=1 FHE_MODUP_FOLD=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_11b.json 2> $O/bench_11b.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 > $O/mehp_00.json 2> $O/mehp_00.err && \
FHE_MODDOWN_FOLD=1 FHE_MODUP_FOLD=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 > $O/mehp_11.json 2> $O/mehp_11.err
