#!/bin/bash
# end-of-round numbers of the side workloads: MEHP24 config 5 and k-way config 4
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/side
mkdir -p $O
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -k 10 600 python bench.py --workload mehp24 --no-cpu-baseline > $O/bench_mehp24.json 2> $O/bench_mehp24.err || { echo "mehp24 failed"; tail -5 $O/bench_mehp24.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_mehp24.json'));print('mehp24', d['ms_per_step'], d.get('max_abs_err'))"
timeout -k 10 600 python bench.py --workload kway --no-cpu-baseline > $O/bench_kway.json 2> $O/bench_kway.err || { echo "kway failed"; tail -5 $O/bench_kway.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_kway.json'));print('kway', d['ms_per_step'], d.get('max_abs_err'))"
echo ALLOK
