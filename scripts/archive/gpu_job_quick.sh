#!/bin/bash
# parity subset (NTT, ops, DirectSort bit-exact, full-size digest) + one bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py -x -q --timeout 600 --timeout-method thread > gpurun_out/tests_quick.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tests_quick.log; exit 1; }
tail -2 gpurun_out/tests_quick.log
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/bench_quick_$i.json 2> gpurun_out/bench_quick.err || { echo "bench failed"; tail -5 gpurun_out/bench_quick.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_quick_$i.json'));r=d['roofline'];print(d['ms_per_step'], r['clocked_ms_per_sort'], r['kernel'], r['frac'], {k:v['avg_us'] for k,v in list(r['kernels_by_caller'].items())[:9]})"
done
echo ALLOK
