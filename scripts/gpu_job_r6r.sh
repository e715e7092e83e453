#!/bin/bash
# round 6 A/B: with the int32-LDS fp64 ModDown kernel (default now), the fp / integer
# switch-over FHE_MODDOWN_FP (min targets; 16 = default, 1 = fp64 everywhere): conversion
# micro timings, then the sort and the k-way network with each, alternated
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_r}
mkdir -p $O
for v in 16 1 16 1; do
  FHE_MODDOWN_FP=$v CONV_TAG=min$v timeout -k 10 120 python scripts/conv_micro.py moddown_rescale32 40,20,16,12,10,8,6 >> $O/micro.jsonl 2>> $O/micro.err || { echo "micro failed"; tail $O/micro.err; exit 1; }
done
cat $O/micro.jsonl
for v in 16 8 1 16 8 1; do
  FHE_MODDOWN_FP=$v timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench.json')); print('sort min=$v', d['ms_per_step'], d.get('max_abs_err'))"
done
for v in 16 1 16 1; do
  FHE_MODDOWN_FP=$v timeout -k 10 200 python bench.py --workload kway --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/kway.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/kway.json')); print('kway min=$v', d['ms_per_step'], d.get('max_abs_err'))"
done
