#!/bin/bash
# round-3 re-entry check: full GPU suite, smoke, default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r3v2}
mkdir -p $O
(while sleep 50; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=20 > $O/tests_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/tests_gpu.log; exit 1; }
tail -25 $O/tests_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print(d['ms_per_step'], d['value'], d.get('max_abs_err'), r['kernel'], r['frac'], r.get('traffic'), r.get('valu_frac'), d.get('cold_sort_s'))"
echo ALLOK
