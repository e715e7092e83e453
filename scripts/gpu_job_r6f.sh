#!/bin/bash
# round 6: fp64 conversions with vector-loaded constants (LDS-staged sources, target pairs) --
# micro A/B at every size, parity with both fp kernels forced
# on, then the sort: default / FHE_MODDOWN_FP=0 / + FHE_MODUP_FP=1
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_f}
mkdir -p $O
for fp in 0 1; do
  FHE_MODDOWN_FP=$fp FHE_MODUP_FP=$fp CONV_TAG=fp$fp timeout -k 10 150 python scripts/conv_micro.py moddown_rescale32,modup32 40,30,24,16,10 >> $O/micro.jsonl 2>> $O/micro.err || { echo "micro failed"; tail $O/micro.err; exit 1; }
done
cat $O/micro.jsonl
FHE_MODDOWN_FP=1 FHE_MODUP_FP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_mehp24.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20; exit 1; }
tail -2 $O/tests.log
for arm in def md0 up1 def md0 up1; do
  case $arm in def) E="";; md0) E="FHE_MODDOWN_FP=0";; up1) E="FHE_MODUP_FP=1";; esac
  env $E timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_$arm.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_$arm.json')); print('$arm', d['ms_per_step'], d.get('max_abs_err'))"
done
