#!/bin/bash
# A/B of env settings with full per-kernel clocks: gpu_job_envab2.sh "VAR=v" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out
i=0
for S in "$@"; do
  i=$((i+1))
  env $S timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --clock-json gpurun_out/envab2_clock_$i.json > gpurun_out/envab2_$i.json 2>gpurun_out/envab2_$i.err || { echo "bench $S failed"; tail -5 gpurun_out/envab2_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/envab2_$i.json'));r=d['roofline'];print('$S', d['ms_per_step'], r['clocked_ms_per_sort'])"
done
echo ALLOK
