#!/bin/bash
# round 5: multi-row twiddle staging + narrow fused blocks -- tests, bench,
# shard rehearsal (per-rank compute at world 1/2/4/8)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_i}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "large_rings or batched or stacked" --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && \
SHARD_CLOCK=$O/shard_clock_w8.json timeout -k 10 600 python scripts/shard_rehearsal.py direct 1 2 4 8 > $O/shard_direct.jsonl 2> $O/shard_direct.err
