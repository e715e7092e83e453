#!/bin/bash
# round 4: one rank's compute at world 1/2/4/8 on the final library (no-op
# all-reduce; scripts/shard_rehearsal.py), the N=1024 sort with 1 and 2 lanes
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r4shard
mkdir -p $O
SHARD_LANES=2,1 timeout -k 10 600 python scripts/shard_rehearsal.py direct 1 2 4 8 > $O/shard_direct.jsonl 2> $O/shard_direct.err || { echo "shard failed"; tail -5 $O/shard_direct.err; exit 1; }
cat $O/shard_direct.jsonl
echo ALLOK
