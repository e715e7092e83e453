#!/bin/bash
# round 3: configs 4 (k-way k=5, N=3125) and 5 (MEHP24 N=4096) benches and
# kernel traces on the current build
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3f
mkdir -p $O
export TMPDIR=/tmp
(while sleep 50; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -k 10 400 python bench.py --workload kway --steps 2 --no-cpu-baseline --clock-json $O/clock_kway.json > $O/bench_kway.json 2> $O/bench_kway.err || { echo "kway bench failed"; tail -20 $O/bench_kway.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_kway.json'));r=d['roofline'];print('kway', d['ms_per_step'], d['value'], d['max_abs_err'], d['hmult_per_sort'], r['kernel'], r['frac'], r['run_op'])"
timeout -k 10 500 python bench.py --workload mehp24 --steps 1 --no-cpu-baseline --clock-json $O/clock_mehp24.json > $O/bench_mehp24.json 2> $O/bench_mehp24.err || { echo "mehp24 bench failed"; tail -20 $O/bench_mehp24.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_mehp24.json'));r=d['roofline'];print('mehp24', d['ms_per_step'], d['value'], d['max_abs_err'], d['hmult_per_sort'], r['kernel'], r['frac'], r['run_op'])"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace_kway" -o run -- python3 "$R/bench.py" --workload kway --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --lanes 1 > $O/trace_kway.log 2>&1 || { echo "kway trace failed"; tail -5 $O/trace_kway.log; exit 1; }
python scripts/trace_summary.py $O/trace_kway/run_kernel_trace.csv > $O/trace_kway_summary.txt && head -30 $O/trace_kway_summary.txt
gzip -f $O/trace_kway/run_kernel_trace.csv
echo ALLOK
