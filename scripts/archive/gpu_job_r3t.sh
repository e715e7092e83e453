#!/bin/bash
# split-exchange 512-point column passes: NTT parity, NTT probe, MEHP24 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3t
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "ntt or ring_2_17 or large_rings or wide_digits" > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python3 scripts/ntt_probe.py > $O/ntt_probe.jsonl 2> $O/ntt_probe.err || { echo "probe failed"; tail -5 $O/ntt_probe.err; exit 1; }
cat $O/ntt_probe.jsonl
timeout -k 10 400 python bench.py --workload mehp24 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_mehp24.json 2> $O/bench_mehp24.err || { echo "bench failed"; tail -5 $O/bench_mehp24.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_mehp24.json'));print('mehp24', d['ms_per_step'], d['value'], d['max_abs_err'])"
echo ALLOK
