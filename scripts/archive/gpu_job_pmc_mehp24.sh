#!/bin/bash
# MEHP24 config-5 GPU test, then the PMC pass that died in round 1, with the
# Python fault handler on (host stack of a SIGSEGV) and a hard time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/pmc_mehp24
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mehp24.py -x -v --timeout 300 --timeout-method thread -k "reference_parameters" > $O/tests.log 2>&1 || { echo "mehp24 tests failed"; tail -30 $O/tests.log; exit 1; }
tail -6 $O/tests.log
(while sleep 50; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_[a-z]' --output-format csv -d "$R/$O/pmc_FETCH_SIZE" -o run -- python3 -X faulthandler "$R/bench.py" --workload mehp24 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --lanes 1 > $O/pmc_FETCH_SIZE.log 2>&1
echo "pmc rc=$?"
tail -40 $O/pmc_FETCH_SIZE.log
