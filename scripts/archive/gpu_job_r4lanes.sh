#!/bin/bash
# round 4: sort wall vs batch lanes per GPU (bench.py --lanes), current library
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r4lanes}
mkdir -p $O
for L in 2 4 3 1; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 4 --mask-steps 0 --lanes $L > $O/lanes_$L.json 2> $O/lanes_$L.err || { echo "lanes $L failed"; tail -5 $O/lanes_$L.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('lanes', sys.argv[2], d['ms_per_step'])" $O/lanes_$L.json $L
done
echo ALLOK
