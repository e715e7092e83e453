#!/bin/bash
# round 5: rotation sums in one pass per 8 terms (Engine::add_many_inplace,
# FHE_ADD_MANY=1 default) -- parity, A/B on the N=1024 sort
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_z}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
FHE_ADD_MANY=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_0.json 2> $O/bench_0.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_1.json 2> $O/bench_1.err && \
FHE_ADD_MANY=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_0b.json 2> $O/bench_0b.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_1b.json 2> $O/bench_1b.err && \
FHE_ADD_MANY=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_0c.json 2> $O/bench_0c.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_1c.json 2> $O/bench_1c.err
