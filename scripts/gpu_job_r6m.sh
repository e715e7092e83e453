#!/bin/bash
# round 6: the multi-rank bench path on the final library -- two ranks sharing the
# one GPU (self-launched, host/gloo exchange: RCCL refuses duplicate devices), the
# N=1024 sort and the k-way replicas
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_m}
mkdir -p $O
timeout -k 10 400 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_g2.json 2> $O/bench_g2.err || { echo "g2 failed"; tail -20 $O/bench_g2.err; exit 1; }
cat $O/bench_g2.json
timeout -k 10 400 python bench.py --gpus 2 --workload kway --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/kway_g2.json 2> $O/kway_g2.err || { echo "kway g2 failed"; tail -20 $O/kway_g2.err; exit 1; }
cat $O/kway_g2.json
