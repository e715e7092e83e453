#!/bin/bash
# GPU parity suite + one bench line with the per-kernel clock (tag = $1, extra bench args after)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 600 python bench.py --no-cpu-baseline --clock-json gpurun_out/clock_$TAG.json "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
echo ALLOK
