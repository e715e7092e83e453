#!/bin/bash
# round 6: ModUp split -- the Q targets on the fp64 kernel, the special primes on
# the 128-bit one (FHE_MODUP_FP=1): micro A/B, parity forced on, sort A/B; then
# the per-kernel clock of one shard-rehearsal rank at world 1 and 8 (one lane)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_g}
mkdir -p $O
for fp in 0 1; do
  FHE_MODUP_FP=$fp CONV_TAG=up$fp timeout -k 10 150 python scripts/conv_micro.py modup32 40,30,24,16 >> $O/micro.jsonl 2>> $O/micro.err || { echo "micro failed"; tail $O/micro.err; exit 1; }
done
cat $O/micro.jsonl
FHE_MODUP_FP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_mehp24.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20; exit 1; }
tail -2 $O/tests.log
for arm in def up1 def up1; do
  case $arm in def) E="";; up1) E="FHE_MODUP_FP=1";; esac
  env $E timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_$arm.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_$arm.json')); print('$arm', d['ms_per_step'], d.get('max_abs_err'))"
done
for w in 1 8; do
  SHARD_LANES=1 SHARD_CLOCK=$O/shard_clock_w$w.json timeout -k 10 300 python scripts/shard_rehearsal.py direct $w >> $O/shard.jsonl 2>> $O/shard.err || { echo "rehearsal failed"; tail $O/shard.err; exit 1; }
done
cat $O/shard.jsonl
