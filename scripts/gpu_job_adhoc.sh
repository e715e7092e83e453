set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "sortutils or n2048 or digest or sign4 or scale59" > gpurun_out/tests_r2c.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/tests_r2c.log; exit 1; }
tail -15 gpurun_out/tests_r2c.log
timeout -k 10 600 python bench.py --no-cpu-baseline --clock-json gpurun_out/clock_r2c.json > gpurun_out/bench_r2c.json 2> gpurun_out/bench_r2c.err || { echo "bench failed"; tail -5 gpurun_out/bench_r2c.err; exit 1; }
cat gpurun_out/bench_r2c.json
