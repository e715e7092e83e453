#!/bin/bash
# round 6: the one-GPU shard rehearsal (rank 0's compute at world 1/2/4/8) with 1-4
# lanes (verdict r5 item 4), after the parity tests the round's NTT-registry /
# fused-kernel assertions touch
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_w}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "large_rings or relin or rotat" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20; exit 1; }
tail -1 $O/tests.log
SHARD_LANES=1,2,3,4 timeout -k 10 600 python scripts/shard_rehearsal.py direct 1 2 4 8 > $O/shard_direct.jsonl 2> $O/shard_direct.err || { echo "rehearsal failed"; tail $O/shard_direct.err; exit 1; }
cat $O/shard_direct.jsonl
