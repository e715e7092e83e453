#!/bin/bash
# parity subset, then short DirectSort benches under env sets:
# gpu_job_envset.sh "A=1 B=0" "A=0 B=0" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py -x -q --timeout 600 --timeout-method thread > gpurun_out/tests_quick.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tests_quick.log; exit 1; }
tail -2 gpurun_out/tests_quick.log
i=0
for V in "$@"; do
  i=$((i+1))
  env $V timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/envset_$i.json 2>gpurun_out/envset_$i.err || { echo "bench $V failed"; tail -5 gpurun_out/envset_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/envset_$i.json'));r=d['roofline'];print('$V', d['ms_per_step'], d['max_abs_err'], {k:(v['avg_us'],v['GBps']) for k,v in list(r['kernels_by_caller'].items())[:12]})"
done
echo ALLOK
