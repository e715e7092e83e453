#!/bin/bash
# lanes x stack A/B over short DirectSort benches: gpu_job_lanes2.sh "3 32" "4 32" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out/lanes2
i=0
for V in "$@"; do
  i=$((i+1)); set -- $V
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 3 --lanes $1 --stack $2 > gpurun_out/lanes2/b_$i.json 2>gpurun_out/lanes2/b_$i.err || { echo "bench $V failed"; tail -5 gpurun_out/lanes2/b_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/lanes2/b_$i.json'));print('lanes/stack $V', d['ms_per_step'], d['max_abs_err'])"
done
echo ALLOK
