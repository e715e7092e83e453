#!/bin/bash
# bench + rocprofv3 kernel trace of one DirectSort (tag = $1, extra bench args after)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- python "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/prof_$TAG.log 2>&1 || { echo "prof failed"; exit 1; }
python scripts/trace_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/prof_$TAG/summary.txt && cat gpurun_out/prof_$TAG/summary.txt && gzip -f gpurun_out/prof_$TAG/run_kernel_trace.csv
echo ALLOK
