#!/bin/bash
# PS node add fused into the tensor pass: parity + benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3aa
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_bootstrap.py tests/test_gpu_mehp24.py > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_direct.json 2> $O/bench_direct.err || { echo "direct failed"; tail -5 $O/bench_direct.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_direct.json'));print('direct', d['ms_per_step'], d['value'], d['max_abs_err'])"
timeout -k 10 300 python3 scripts/boot_prof.py > $O/boot.log 2>&1 || { echo "boot failed"; tail -5 $O/boot.log; exit 1; }
cat $O/boot.log
echo ALLOK
