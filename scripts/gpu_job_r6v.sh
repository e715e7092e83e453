#!/bin/bash
# round 6 A/B: the HMult-tail / key-switch-finish FP rows loading their epilogue operands
# in the store loop (lib/ab_mt0.so, -DFHE_NTT_FP_EPI_PRE_MT=0: 164 -> 97 VGPRs, 3 -> 4
# waves per SIMD) against before the butterflies (lib/libfhesort.so): N=1024 sorts and
# MEHP24 alternated, then one kernel trace of a sort with each
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6_v}
mkdir -p $O
lib() { if [ $1 = def ]; then echo $R/fhe-sorting_amd/lib/libfhesort.so; else echo $R/fhe-sorting_amd/lib/ab_$1.so; fi; }
for v in def mt0 def mt0 def mt0; do
  FHE_LIB=$(lib $v) timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench.json')); print('sort $v', d['ms_per_step'], d.get('max_abs_err'))" | tee -a $O/ab.txt
done
for v in def mt0 def mt0; do
  FHE_LIB=$(lib $v) timeout -k 10 240 python bench.py --workload mehp24 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/mehp24.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/mehp24.json')); print('mehp24 $v', d['ms_per_step'], d.get('max_abs_err'))" | tee -a $O/ab.txt
done
for v in def mt0; do
  FHE_LIB=$(lib $v) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/prof_$v.log 2>&1 || { echo "prof failed"; tail $O/prof_$v.log; exit 1; }
done
find $O -name "*kernel_stats.csv" | head
