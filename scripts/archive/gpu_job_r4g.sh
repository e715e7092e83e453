#!/bin/bash
# round 4: MEHP24 (config 5) and k-way (config 4) bench lines on the current
# build, each with its roofline (MEHP24: the per-phase kernel / op-level byte
# split, roofline.phases) and CPU baseline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r4g}
mkdir -p $O
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
export ROC_AQL_QUEUE_SIZE=131072
timeout -k 10 900 python bench.py --workload mehp24 --steps 1 --warmup 1 --clock-json $O/clock_mehp24.json > $O/bench_mehp24.json 2> $O/bench_mehp24.err || { echo "mehp24 failed"; tail -5 $O/bench_mehp24.err; exit 1; }
python - $O/bench_mehp24.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d.get('roofline') or {}
print('mehp24', d['sort_seconds'], 'err', d['max_abs_err'], 'run_op', (r.get('run_op') or {}).get('frac'), 'run', r.get('run', {}).get('frac'))
for k, v in (r.get('phases') or {}).items(): print('  ', k, v)
PY
timeout -k 10 600 python bench.py --workload kway --steps 2 --warmup 1 > $O/bench_kway.json 2> $O/bench_kway.err || { echo "kway failed"; tail -5 $O/bench_kway.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('kway', d['ms_per_step'], d.get('max_abs_err'))" $O/bench_kway.json
echo ALLOK
