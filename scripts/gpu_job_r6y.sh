#!/bin/bash
# round 6 closing: the one-GPU shard rehearsal (rank 0's compute at world 1/2/4/8,
# the default two lanes) on the final library
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_y}
mkdir -p $O
SHARD_LANES=2 timeout -k 10 600 python scripts/shard_rehearsal.py direct 1 2 4 8 > $O/shard_direct.jsonl 2> $O/shard_direct.err || { echo "rehearsal failed"; tail $O/shard_direct.err; exit 1; }
cat $O/shard_direct.jsonl
