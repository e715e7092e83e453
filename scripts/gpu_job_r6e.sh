#!/bin/bash
# round 6: fp64 ModDown + rescale, targets per work item 2 / 4 (FHE_CONV_TPI):
# micro A/B, parity with the fp kernel forced at every size, sort and MEHP24 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_e}
mkdir -p $O
for arm in "0 2" "1 2" "1 4"; do
  set -- $arm
  FHE_MODDOWN_FP=$1 FHE_CONV_TPI=$2 CONV_TAG=fp$1_tpi$2 timeout -k 10 150 python scripts/conv_micro.py moddown_rescale32 40,30,24,16 >> $O/micro.jsonl 2>> $O/micro.err || { echo "micro failed"; tail $O/micro.err; exit 1; }
done
cat $O/micro.jsonl
FHE_MODDOWN_FP=1 FHE_CONV_TPI=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_mehp24.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20; exit 1; }
tail -2 $O/tests.log
for arm in def md0 tpi4 def md0 tpi4; do
  case $arm in def) E="";; md0) E="FHE_MODDOWN_FP=0";; tpi4) E="FHE_CONV_TPI=4";; esac
  env $E timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_$arm.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_$arm.json')); print('$arm', d['ms_per_step'], d.get('max_abs_err'))"
done
for arm in def md0; do
  case $arm in def) E="";; md0) E="FHE_MODDOWN_FP=0";; esac
  env $E timeout -k 10 300 python bench.py --workload mehp24 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/mehp_$arm.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/mehp_$arm.json')); print('mehp24 $arm', d['ms_per_step'], d.get('max_abs_err'))"
done
