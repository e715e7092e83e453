#!/bin/bash
# k-way phase split (FHE_KWAY_TIMES) and the bootstrap stage times + counters
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 300 python scripts/boot_stages.py 16 4096 > $O/boot_stages.json 2> $O/boot_stages.err || { echo "boot stages failed"; tail -5 $O/boot_stages.err; exit 1; }
cat $O/boot_stages.json
FHE_KWAY_TIMES=1 timeout -k 10 400 python bench.py --workload kway --steps 1 --no-cpu-baseline --no-roofline > $O/kway_times.json 2> $O/kway_times.err || { echo "kway failed"; tail -5 $O/kway_times.err; exit 1; }
grep -v "^\[Gloo\]" $O/kway_times.err | tail -30
echo ALLOK
