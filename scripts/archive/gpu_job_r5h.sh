#!/bin/bash
# round 5: shard rehearsal with the per-phase clock at world 8 (verdict r4
# item 7), and the corrected 16-B access-pattern probe
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_h}
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/row_pattern.hip -o /tmp/rp 2>/dev/null && \
timeout -k 10 120 /tmp/rp > $O/row_pattern.jsonl && \
SHARD_CLOCK=$O/shard_clock_w8.json timeout -k 10 600 python scripts/shard_rehearsal.py direct 1 2 4 8 > $O/shard_direct.jsonl 2> $O/shard_direct.err
