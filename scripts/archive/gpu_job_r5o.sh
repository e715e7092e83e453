#!/bin/bash
# round 5: leaf-sum passes of up to 32 leaves (FHE_PS_CHUNK=32) vs 16 (default) --
# parity (MFMA, digests, parity, k-way, bootstrap), A/B on the N=1024 sort and MEHP24
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_o}
mkdir -p $O
FHE_PS_CHUNK=32 timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_digests.py tests/test_gpu_parity.py tests/test_gpu_kway.py tests/test_gpu_bootstrap.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
FHE_PS_CHUNK=16 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_16.json 2> $O/bench_16.err && \
FHE_PS_CHUNK=32 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_32.json 2> $O/bench_32.err && \
FHE_PS_CHUNK=16 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_16b.json 2> $O/bench_16b.err && \
FHE_PS_CHUNK=32 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_32b.json 2> $O/bench_32b.err && \
FHE_PS_CHUNK=16 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 > $O/mehp_16.json 2> $O/mehp_16.err && \
FHE_PS_CHUNK=32 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 > $O/mehp_32.json 2> $O/mehp_32.err
