#!/bin/bash
# round 3: bench the OpenFHE split at 40 bits against the round-2 spec, and the
# self-launched two-rank bench on one GPU
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --clock-json $O/clock_of40.json > $O/bench_of40.json 2> $O/bench_of40.err || { echo "bench of40 failed"; tail -20 $O/bench_of40.err; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --scale-bits 50 --ps-split engine > $O/bench_en50.json 2> $O/bench_en50.err || { echo "bench en50 failed"; tail -20 $O/bench_en50.err; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --ps-split engine --no-roofline > $O/bench_en40.json 2> $O/bench_en40.err || { echo "bench en40 failed"; tail -20 $O/bench_en40.err; exit 1; }
for f in of40 en50 en40; do python -c "
import json; d=json.load(open('$O/bench_$f.json')); r=d.get('roofline') or {}
print('$f', d['ms_per_step'], d['value'], d['max_abs_err'], d['hmult_per_sort'], d['cold_sort_s'], d['config']['special_primes'], r.get('kernel'), r.get('frac'), (r.get('run_op') or {}).get('frac_over_wall'))"; done
timeout -k 10 400 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_2rank.json 2> $O/bench_2rank.err || { echo "2-rank bench failed"; tail -20 $O/bench_2rank.err; exit 1; }
cat $O/bench_2rank.json
echo ALLOK
