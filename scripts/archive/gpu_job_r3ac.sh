#!/bin/bash
# fp64 linear sums A/B on one box (FHE_LIN_FP64 = 1 / 0 / 1)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3ac
mkdir -p $O
for M in 1 0 1 0; do
  FHE_LIN_FP64=$M timeout -k 10 300 python bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-roofline --clock-json $O/clock_$M.json > $O/bench_direct_$M.json 2> $O/bench_direct_$M.err || { echo "direct failed"; tail -5 $O/bench_direct_$M.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_direct_$M.json'));print('FP64=$M direct', d['ms_per_step'], d['max_abs_err'])"
done
echo ALLOK
