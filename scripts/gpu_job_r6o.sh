#!/bin/bash
# round 6: conversions chunked by >= 8 targets on narrow launches (was >= 4):
# config 4, the N=1024 sort and the world-8 rehearsal, against FHE_CONV_CHUNK=4
# forced... (the old rule is not reachable by env: the sweep's fixed chunks bracket it)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_o}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kway.py tests/test_gpu_bootstrap.py -x -q --timeout 300 --timeout-method thread -k "bit_exact or oracle" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  timeout -k 10 200 python bench.py --workload kway --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/kway_$rep.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json; d=json.load(open('$O/kway_$rep.json')); print('kway', $rep, d['ms_per_step'], d.get('max_abs_err'))"
  timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-roofline > $O/sort_$rep.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json; d=json.load(open('$O/sort_$rep.json')); print('sort', $rep, d['ms_per_step'], d.get('max_abs_err'))"
done
SHARD_LANES=2 timeout -k 10 400 python scripts/shard_rehearsal.py direct 1 8 > $O/shard.jsonl 2>> $O/shard.err && cat $O/shard.jsonl
