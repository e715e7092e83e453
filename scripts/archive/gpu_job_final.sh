#!/bin/bash
# round-end rehearsal: full GPU suite, smoke(), default bench (what the driver runs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/final
mkdir -p $O
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/tests_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/tests_gpu.log; exit 1; }
tail -2 $O/tests_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
echo ALLOK
