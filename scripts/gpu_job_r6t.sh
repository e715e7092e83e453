#!/bin/bash
# round 6: same-box A/B of the round's closing libraries -- lib/ab_old.so (kernels.hip of
# daf6091, the 45acad0f library) against lib/libfhesort.so (int32 ModDown sources, fp64
# ModDown everywhere): N=1024 sorts, alternated
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_t}
mkdir -p $O
for v in old new old new old new; do
  L=$R/fhe-sorting_amd/lib/libfhesort.so; [ $v = old ] && L=$R/fhe-sorting_amd/lib/ab_old.so
  FHE_LIB=$L timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench.json')); print('sort $v', d['ms_per_step'], d.get('max_abs_err'))" | tee -a $O/ab.txt
done
