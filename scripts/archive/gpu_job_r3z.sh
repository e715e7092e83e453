#!/bin/bash
# DirectSort lanes x stack sweep
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3z
mkdir -p $O
for LS in "2 32" "3 32" "4 32" "3 16" "4 16" "6 16" "8 8"; do
  set -- $LS
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline --lanes $1 --stack $2 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { echo "bench $1 $2 failed"; tail -5 $O/b_$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_$1_$2.json'));print('lanes $1 stack $2', d['ms_per_step'], d['hbm_peak_gb_rank0'])"
done
echo ALLOK
