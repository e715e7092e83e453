#!/bin/bash
# FHE_NTT_FULL A/B (exact-grid variants of the lift column / rescale row / inverse row passes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3y
mkdir -p $O
for M in 181 183 189 245 255; do
  FHE_NTT_FULL=$M timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_direct_$M.json 2> $O/bench_direct_$M.err || { echo "direct failed"; tail -5 $O/bench_direct_$M.err; exit 1; }
  FHE_NTT_FULL=$M timeout -k 10 400 python bench.py --workload mehp24 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_mehp24_$M.json 2> $O/bench_mehp24_$M.err || { echo "mehp24 failed"; tail -5 $O/bench_mehp24_$M.err; exit 1; }
  python -c "import json;a=json.load(open('$O/bench_direct_$M.json'));b=json.load(open('$O/bench_mehp24_$M.json'));print('FULL=$M direct', a['ms_per_step'], 'mehp24', b['ms_per_step'], a['max_abs_err'], b['max_abs_err'])"
done
echo ALLOK
