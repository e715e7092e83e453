#!/bin/bash
# round 3: parity/wire/collective subset after the encoder + sampler changes,
# the default bench with the cold-sort breakdown, then the MEHP24 PMC pass
# that aborted in round 2, with the engine's fault report on (launch notes,
# faulting PC / address and the maps lines that hold them)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wire.py tests/test_gpu_collective.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['ms_per_step'], d['cold_sort_s'], d['cold_breakdown'], d['timed_host_costs'], d['max_abs_err'], d['roofline']['kernel'], d['roofline']['frac'])"
(while sleep 50; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
FHE_FAULT_REPORT=1 timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_[a-z]' --output-format csv -d "$R/$O/pmc_FETCH_SIZE" -o run -- python3 "$R/bench.py" --workload mehp24 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --lanes 1 > $O/pmc_FETCH_SIZE.log 2>&1
echo "pmc rc=$?"
grep -A12 "fhe fault report\] SIG" $O/pmc_FETCH_SIZE.log | head -40
tail -5 $O/pmc_FETCH_SIZE.log
