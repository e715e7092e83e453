#!/bin/bash
# MEHP24 (config 5) bench under env settings: gpu_job_mehp.sh "VAR=v" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out
i=0
for S in "$@"; do
  i=$((i+1))
  env $S timeout -k 10 600 python bench.py --workload mehp24 --no-cpu-baseline > gpurun_out/mehp_$i.json 2> gpurun_out/mehp_$i.err || { echo "bench $S failed"; tail -5 gpurun_out/mehp_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/mehp_$i.json'));r=d['roofline'];print('$S', d['ms_per_step'], d['max_abs_err'], {k:(v['avg_us'],v['GBps']) for k,v in list(r['kernels'].items())[:6]})"
done
echo ALLOK
