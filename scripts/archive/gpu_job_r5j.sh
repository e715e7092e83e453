#!/bin/bash
# round 5: small integer launches on an auxiliary stream -- parity, bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_j}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
FHE_NTT_AUX=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_aux0.json 2> $O/bench_aux0.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_aux1.json 2> $O/bench_aux1.err && \
FHE_NTT_AUX=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_aux0b.json 2> $O/bench_aux0b.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_aux1b.json 2> $O/bench_aux1b.err
