#!/bin/bash
# double-hoisted BSGS (babies over QP): bootstrap + k-way parity, times
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3r
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bootstrap.py tests/test_gpu_kway.py > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python3 scripts/boot_prof.py > $O/boot.log 2>&1 || { echo "boot failed"; tail -5 $O/boot.log; exit 1; }
cat $O/boot.log
FHE_KWAY_TIMES=1 timeout -k 10 400 python bench.py --workload kway --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_kway.json 2> $O/bench_kway.err || { echo "kway failed"; tail -5 $O/bench_kway.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_kway.json'));print('kway', d['ms_per_step'], d['value'], d['max_abs_err'])"
grep "k-way" $O/bench_kway.err | tail -3
echo ALLOK
