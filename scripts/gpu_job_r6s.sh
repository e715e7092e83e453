#!/bin/bash
# round 6 A/B: the fp64 ModUp kernel with int32 sources in LDS (FHE_MODUP_FP = min
# sources; 0 = off, the default so far): micro timings, parity under 1, the sort and
# MEHP24 with each, alternated
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_s}
mkdir -p $O
for v in 0 1 0 1; do
  FHE_MODUP_FP=$v CONV_TAG=up$v timeout -k 10 120 python scripts/conv_micro.py modup32 40,30,20,10 >> $O/micro.jsonl 2>> $O/micro.err || { echo "micro failed"; tail $O/micro.err; exit 1; }
done
cat $O/micro.jsonl
FHE_MODUP_FP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_mehp24.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20; exit 1; }
tail -2 $O/tests.log
for v in 0 1 0 1; do
  FHE_MODUP_FP=$v timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench.json')); print('sort up=$v', d['ms_per_step'], d.get('max_abs_err'))"
done
for v in 0 1 0 1; do
  FHE_MODUP_FP=$v timeout -k 10 240 python bench.py --workload mehp24 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/mehp24.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/mehp24.json')); print('mehp24 up=$v', d['ms_per_step'], d.get('max_abs_err'))"
done
