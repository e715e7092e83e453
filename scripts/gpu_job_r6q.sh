#!/bin/bash
# round 6 A/B: FHE_MDFP_I32 on BASELINE config 5 (MEHP24, the K = 16 ModDown kernel,
# 2 -> 4 waves per SIMD), two sorts each, alternated
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_q}
mkdir -p $O
for v in 0 1 0 1; do
  FHE_MDFP_I32=$v timeout -k 10 240 python bench.py --workload mehp24 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/mehp24_$v.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/mehp24_$v.json')); print('i32=$v', d['ms_per_step'], d.get('max_abs_err'))"
done
