#!/bin/bash
# round 5: the one-GPU shard rehearsal (rank 0's compute at world 1/2/4/8) on the
# final library
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_w}
mkdir -p $O
timeout -k 10 600 python scripts/shard_rehearsal.py direct 1 2 4 8 > $O/shard_direct.jsonl 2> $O/shard_direct.err
