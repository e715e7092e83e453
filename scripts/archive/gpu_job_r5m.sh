#!/bin/bash
# round 5: row-pass twiddles staged in dynamic LDS for every register-only row
# pass (FHE_NTT_TWL_ROWS=16, default) vs blocks of >= 4 segments only (=4):
# parity (k-way and bootstrap included), A/B on the three benched workloads
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_m}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_kway.py tests/test_gpu_bootstrap.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
FHE_NTT_TWL_ROWS=4 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload kway > $O/kway_4.json 2> $O/kway_4.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload kway > $O/kway_16.json 2> $O/kway_16.err && \
FHE_NTT_TWL_ROWS=4 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_4.json 2> $O/bench_4.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_16.json 2> $O/bench_16.err && \
FHE_NTT_TWL_ROWS=4 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 > $O/mehp_4.json 2> $O/mehp_4.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 > $O/mehp_16.json 2> $O/mehp_16.err && \
FHE_NTT_TWL_ROWS=8 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload kway > $O/kway_8.json 2> $O/kway_8.err && \
FHE_NTT_TWL_ROWS=4 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_4b.json 2> $O/bench_4b.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_16b.json 2> $O/bench_16b.err
