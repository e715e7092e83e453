#!/bin/bash
# round 5: the full GPU suite and smoke() with the folded leaf sums and 32-leaf
# passes on by default, then MEHP24 and k-way benches (regression check)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_q}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 > $O/mehp.json 2> $O/mehp.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload kway > $O/kway.json 2> $O/kway.err && \
echo ALLOK
