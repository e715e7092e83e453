#!/bin/bash
# round 6 A/B: the fp64 ModDown kernel's LDS sources as int32 pairs (FHE_MDFP_I32=1,
# half the LDS, 56 VGPRs / 7 waves) against double pairs (0): conversion micro
# timings, parity under 1, then the N=1024 sort with each form
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_p}
mkdir -p $O
for v in 0 1 0 1; do
  FHE_MDFP_I32=$v CONV_TAG=i32_$v timeout -k 10 120 python scripts/conv_micro.py moddown_rescale32 40,30,20,10 >> $O/micro.jsonl 2>> $O/micro.err || { echo "micro failed"; tail $O/micro.err; exit 1; }
done
cat $O/micro.jsonl
FHE_MDFP_I32=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_mehp24.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20; exit 1; }
tail -2 $O/tests.log
for v in 0 1 0 1; do
  FHE_MDFP_I32=$v timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_$v.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_$v.json')); print('i32=$v', d['ms_per_step'], d.get('max_abs_err'))"
done
