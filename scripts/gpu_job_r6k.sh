#!/bin/bash
# round 6: the fused key switch for stacks of fewer than 4 members (FHE_KS_FUSE_MIN
# = 1 / 4): parity with it forced at one member, the world-8 / world-4 rehearsal
# and config 4 (one-ciphertext ops)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_k}
mkdir -p $O
FHE_KS_FUSE_MIN=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bootstrap.py tests/test_gpu_kway.py -x -q --timeout 300 --timeout-method thread -k "large_rings or bit_exact or config" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20; exit 1; }
tail -2 $O/tests.log
for m in 1 4; do
  FHE_KS_FUSE_MIN=$m SHARD_LANES=2 timeout -k 10 400 python scripts/shard_rehearsal.py direct 1 4 8 > $O/shard_min$m.jsonl 2>> $O/shard.err || { echo "rehearsal failed"; tail $O/shard.err; exit 1; }
  echo "min $m"; cat $O/shard_min$m.jsonl
done
for m in 1 4; do
  FHE_KS_FUSE_MIN=$m timeout -k 10 300 python bench.py --workload kway --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/kway_min$m.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json; d=json.load(open('$O/kway_min$m.json')); print('kway min $m', d['ms_per_step'], d.get('max_abs_err'))"
done
