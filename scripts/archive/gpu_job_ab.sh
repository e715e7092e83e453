#!/bin/bash
# A/B of an env switch over short DirectSort benches: gpu_job_ab.sh VAR v1 v2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out
VAR=$1; shift
for V in "$@"; do
  env $VAR=$V timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/ab_${VAR}_$V.json 2>gpurun_out/ab_${VAR}_$V.err || { echo "bench $V failed"; tail -5 gpurun_out/ab_${VAR}_$V.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_${VAR}_$V.json'));r=d['roofline'];print('$VAR=$V', d['ms_per_step'], d['max_abs_err'], {k:(v['avg_us'],v['GBps']) for k,v in list(r['kernels_by_caller'].items())[:10]})"
done
