#!/bin/bash
# round 5: the reference CLI context test (ring 2^17, depth 44, testcase.json),
# then the config-4 / config-5 benches with the FP NTT
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_d}
mkdir -p $O
df -h /tmp . > $O/df.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_wire.py -x -v -s --timeout 500 --timeout-method thread > $O/wire.log 2>&1 ; echo "wire rc $?" >> $O/wire.log
timeout -k 10 400 python bench.py --workload mehp24 > $O/bench_mehp24.json 2> $O/bench_mehp24.err && \
timeout -k 10 400 python bench.py --workload kway > $O/bench_kway.json 2> $O/bench_kway.err
