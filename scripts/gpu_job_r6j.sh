#!/bin/bash
# round 6: with the integer targets fused (new default), re-check the engine's
# remaining A/B switches on the sort, and MEHP24 with / without the new fusion
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_j}
mkdir -p $O
for rep in 1 2; do
for arm in def shfl29 full255 aux1 stack16 lanes3 twl8; do
  A=""; E="FHE_X=0"
  case $arm in shfl29) E="FHE_NTT_ROW_SHFL=29";; full255) E="FHE_NTT_FULL=255";; aux1) E="FHE_NTT_AUX=1";; stack16) A="--stack 16";; lanes3) A="--lanes 3";; twl8) E="FHE_NTT_TWL_ROWS=8";; esac
  env $E timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-roofline $A > $O/bench_${arm}_$rep.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_${arm}_$rep.json')); print('$arm', $rep, d['ms_per_step'], d.get('max_abs_err'))"
done
done
for arm in def int0; do
  case $arm in def) E="FHE_X=0";; int0) E="FHE_KS_FUSE_INT=0";; esac
  env $E timeout -k 10 300 python bench.py --workload mehp24 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/mehp_$arm.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json; d=json.load(open('$O/mehp_$arm.json')); print('mehp24 $arm', d['ms_per_step'], d.get('max_abs_err'))"
done
