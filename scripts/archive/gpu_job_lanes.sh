#!/bin/bash
# lanes / stack sweep of the headline bench: gpu_job_lanes.sh "lanes stack" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out
i=0
for S in "$@"; do
  i=$((i+1)); set -- $S
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 4 --lanes $1 --stack $2 > gpurun_out/lanes_$i.json 2>gpurun_out/lanes_$i.err || { echo "bench $S failed"; tail -5 gpurun_out/lanes_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/lanes_$i.json'));print('lanes/stack $S', d['ms_per_step'], d['hbm_peak_gb_rank0'])"
done
echo ALLOK
