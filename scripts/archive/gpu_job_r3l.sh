#!/bin/bash
# MEHP24 digit count A/B (dnum 3, 4, 5)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3l
mkdir -p $O
for D in 3 4 5; do
  timeout -k 10 300 python bench.py --workload mehp24 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --dnum $D > $O/bench_d$D.json 2> $O/bench_d$D.err || { echo "bench $D failed"; tail -5 $O/bench_d$D.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_d$D.json'));print($D, d['ms_per_step'], d['max_abs_err'], d['hbm_peak_gb_rank0'])"
done
echo ALLOK
