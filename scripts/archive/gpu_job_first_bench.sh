#!/bin/bash
# First end-to-end GPU session: smoke, N=128 bench, rocprofv3 stats, N=1024 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python bench.py --n-sort 128 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench128.json 2> gpurun_out/bench128.err || { echo "bench128 failed"; exit 1; }
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof128" -o run -- python "$R/bench.py" --n-sort 128 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof128.log 2>&1 || { echo "prof failed"; exit 1; }
timeout -k 10 600 python bench.py --steps 1 --warmup 1 > gpurun_out/bench1024.json 2> gpurun_out/bench1024.err || { echo "bench1024 failed"; exit 1; }
echo ALLOK
