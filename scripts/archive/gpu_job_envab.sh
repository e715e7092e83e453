#!/bin/bash
# A/B of env settings over short DirectSort benches: gpu_job_envab.sh "VAR=v ..." "VAR=w ..." ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out
i=0
for S in "$@"; do
  i=$((i+1))
  env $S timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/envab_$i.json 2>gpurun_out/envab_$i.err || { echo "bench $S failed"; tail -5 gpurun_out/envab_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/envab_$i.json'));r=d['roofline'];print('$S', d['ms_per_step'], r['clocked_ms_per_sort'], {k:v['avg_us'] for k,v in list(r['kernels_by_caller'].items())[:9]})"
done
echo ALLOK
