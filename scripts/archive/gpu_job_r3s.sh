#!/bin/bash
# shard rehearsal (rank 0 of world 1/2/4/8, no-op all-reduce) on the round-3 engine
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3s
mkdir -p $O
timeout -k 10 300 python3 scripts/shard_rehearsal.py direct 1 2 4 8 > $O/shard_direct.jsonl 2> $O/shard_direct.err || { echo "direct failed"; tail -5 $O/shard_direct.err; exit 1; }
cat $O/shard_direct.jsonl
timeout -k 10 500 python3 scripts/shard_rehearsal.py mehp24 1 2 4 8 > $O/shard_mehp24.jsonl 2> $O/shard_mehp24.err || { echo "mehp24 failed"; tail -5 $O/shard_mehp24.err; exit 1; }
cat $O/shard_mehp24.jsonl
echo ALLOK
