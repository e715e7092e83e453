#!/bin/bash
# round-4 first box call: the new / changed GPU tests, then the sort-only profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r4a
mkdir -p $O
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mfma.py tests/test_gpu_wire.py "tests/test_gpu_parity.py::test_ps_split_change_reaches_cached_lanes" tests/test_gpu_collective.py tests/test_gpu_distributed.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
kill $TICK 2>/dev/null
bash scripts/gpu_job_r4prof.sh r4_base
