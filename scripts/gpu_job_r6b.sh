#!/bin/bash
# round 6: fp64 conversions (LDS-staged sources, target pairs) -- micro A/B, parity, sort A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_b}
mkdir -p $O
for fp in 0 1; do
  FHE_MODDOWN_FP=$fp FHE_MODUP_FP=$fp CONV_TAG=fp$fp timeout -k 10 150 python scripts/conv_micro.py moddown_rescale32,modup32 40,30,20,10 >> $O/micro.jsonl 2>> $O/micro.err || { echo "micro failed"; tail $O/micro.err; exit 1; }
done
cat $O/micro.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_mehp24.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20; exit 1; }
tail -2 $O/tests.log
for fp in 0 1 0 1; do
  FHE_MODDOWN_FP=$fp FHE_MODUP_FP=$fp timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_fp$fp.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_fp$fp.json')); print('fp$fp', d['ms_per_step'], d.get('max_abs_err'))"
done
