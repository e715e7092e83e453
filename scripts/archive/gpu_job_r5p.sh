#!/bin/bash
# round 5: leaf sums -- the folded-constant kernel (FHE_LEAF_FOLD=1) and 4 column
# tiles per wave on the window kernel (lib/ab_nc4.so) against the window kernel,
# all with 32-leaf passes: MFMA/digest/parity tests, A/B on the N=1024 sort
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_p}
mkdir -p $O
export FHE_PS_CHUNK=32
FHE_LEAF_FOLD=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_digests.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity_fold.log 2>&1 && \
FHE_LIB=fhe-sorting_amd/lib/ab_nc4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_digests.py -x -q --timeout 300 --timeout-method thread > $O/parity_nc4.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_nc2.json 2> $O/bench_nc2.err && \
FHE_LEAF_FOLD=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_fold.json 2> $O/bench_fold.err && \
FHE_LIB=fhe-sorting_amd/lib/ab_nc4.so timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_nc4.json 2> $O/bench_nc4.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_nc2b.json 2> $O/bench_nc2b.err && \
FHE_LEAF_FOLD=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_foldb.json 2> $O/bench_foldb.err && \
FHE_LEAF_FOLD=1 FHE_PS_CHUNK=16 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_fold16.json 2> $O/bench_fold16.err
