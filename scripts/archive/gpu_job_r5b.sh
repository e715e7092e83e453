#!/bin/bash
# round 5: row-pass access-pattern probe + FP row waves-per-EU A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_b}
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/row_pattern.hip -o /tmp/row_pattern 2>/dev/null && \
timeout -k 10 120 /tmp/row_pattern > $O/row_pattern.jsonl && \
timeout -k 10 300 python bench.py > $O/bench_base.json 2> $O/bench_base.err && \
FHE_LIB=fhe-sorting_amd/lib/ab_fpw4.so timeout -k 10 300 python bench.py > $O/bench_fpw4.json 2> $O/bench_fpw4.err && \
FHE_LIB=fhe-sorting_amd/lib/ab_fpw5.so timeout -k 10 300 python bench.py > $O/bench_fpw5.json 2> $O/bench_fpw5.err
