#!/bin/bash
# ks_inner member groups of 4 vs 8: MEHP24 and DirectSort
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3u
mkdir -p $O
for M in 4 8; do
  FHE_KS_MC=$M timeout -k 10 400 python bench.py --workload mehp24 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_mehp24_$M.json 2> $O/bench_mehp24_$M.err || { echo "bench failed"; tail -5 $O/bench_mehp24_$M.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_mehp24_$M.json'));print('mehp24 MC=$M', d['ms_per_step'], d['max_abs_err'])"
  FHE_KS_MC=$M timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_direct_$M.json 2> $O/bench_direct_$M.err || { echo "direct failed"; tail -5 $O/bench_direct_$M.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_direct_$M.json'));print('direct MC=$M', d['ms_per_step'], d['max_abs_err'])"
done
echo ALLOK
