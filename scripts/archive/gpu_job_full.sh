#!/bin/bash
# full GPU suite, then the default bench, then optional A/B values of FHE_NTT_ROW_SHFL
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/tests_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/tests_gpu.log; exit 1; }
tail -3 gpurun_out/tests_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed"; tail -5 gpurun_out/bench_default.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));r=d['roofline'];print('default', d['ms_per_step'], d['max_abs_err'], r['kernel'], r['frac'], {k:(v['avg_us'],v['GBps']) for k,v in list(r['kernels_by_caller'].items())[:10]})"
for V in "$@"; do
  FHE_NTT_ROW_SHFL=$V timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/ab_shfl_$V.json 2>gpurun_out/ab_shfl_$V.err || { echo "bench $V failed"; tail -5 gpurun_out/ab_shfl_$V.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_shfl_$V.json'));r=d['roofline'];print('SHFL=$V', d['ms_per_step'], {k:(v['avg_us'],v['GBps']) for k,v in list(r['kernels_by_caller'].items())[:10]})"
done
echo ALLOK
