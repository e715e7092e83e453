#!/bin/bash
# wide digits (OpenFHE's dnum 3 for MEHP24): parity, MEHP24 suites, config-5 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "wide_digits or ring_2_17 or modup" > $O/parity.log 2>&1 || { echo "parity failed"; tail -30 $O/parity.log; exit 1; }
tail -8 $O/parity.log
timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_mehp24.py > $O/mehp24.log 2>&1 || { echo "mehp24 failed"; tail -30 $O/mehp24.log; exit 1; }
tail -12 $O/mehp24.log
timeout -k 10 400 python bench.py --workload mehp24 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_mehp24.json 2> $O/bench_mehp24.err || { echo "bench failed"; tail -5 $O/bench_mehp24.err; exit 1; }
cat $O/bench_mehp24.json
echo ALLOK
