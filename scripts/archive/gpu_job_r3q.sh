#!/bin/bash
# fused ModUp row pass + relinearisation: parity, HMult A/B, benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3q
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_digests.py > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
for M in 0 1; do
  FHE_MODUP_KS=$M timeout -k 10 300 python3 scripts/batch_probe.py > $O/probe_$M.log 2>&1 || { echo "probe failed"; tail -5 $O/probe_$M.log; exit 1; }
  echo "FHE_MODUP_KS=$M"; head -9 $O/probe_$M.log
  FHE_MODUP_KS=$M timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_direct_$M.json 2> $O/bench_direct_$M.err || { echo "direct failed"; tail -5 $O/bench_direct_$M.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_direct_$M.json'));print('direct', d['ms_per_step'], d['value'], d['max_abs_err'])"
  FHE_MODUP_KS=$M timeout -k 10 400 python bench.py --workload kway --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_kway_$M.json 2> $O/bench_kway_$M.err || { echo "kway failed"; tail -5 $O/bench_kway_$M.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_kway_$M.json'));print('kway', d['ms_per_step'], d['value'], d['max_abs_err'])"
done
echo ALLOK
