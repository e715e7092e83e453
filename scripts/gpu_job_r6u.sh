#!/bin/bash
# round 6 A/B: targets per work item of the int32-source fp64 ModDown kernel
# (FHE_CONV_TPI = 2, the default, or 4: the int32 -> fp64 conversions of a source
# amortised over 16 FMAs instead of 8, 109 VGPRs / 4 waves): micro timings, the sort
# and MEHP24, alternated
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_u}
mkdir -p $O
for v in 2 4 2 4; do
  FHE_CONV_TPI=$v CONV_TAG=tpi$v timeout -k 10 120 python scripts/conv_micro.py moddown_rescale32 40,20,10 >> $O/micro.jsonl 2>> $O/micro.err || { echo "micro failed"; tail $O/micro.err; exit 1; }
done
cat $O/micro.jsonl
for v in 2 4 2 4; do
  FHE_CONV_TPI=$v timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench.json')); print('sort tpi=$v', d['ms_per_step'], d.get('max_abs_err'))"
done
for v in 2 4 2 4; do
  FHE_CONV_TPI=$v timeout -k 10 240 python bench.py --workload mehp24 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/mehp24.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/mehp24.json')); print('mehp24 tpi=$v', d['ms_per_step'], d.get('max_abs_err'))"
done
