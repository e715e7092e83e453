#!/bin/bash
# round 5: fused relinearisation with the D = 1 streaming store and the digit
# accumulators initialised ahead of the loop (fewer VGPRs) -- parity, A/B vs the
# closing-profile library (lib/ab_old.so) on the N=1024 sort, config 5, world 8
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_l}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
FHE_LIB=fhe-sorting_amd/lib/ab_old.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_old.json 2> $O/bench_old.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_new.json 2> $O/bench_new.err && \
FHE_LIB=fhe-sorting_amd/lib/ab_old.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_old2.json 2> $O/bench_old2.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > $O/bench_new2.json 2> $O/bench_new2.err && \
FHE_LIB=fhe-sorting_amd/lib/ab_old.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 --steps 2 --warmup 1 > $O/mehp_old.json 2> $O/mehp_old.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --workload mehp24 --steps 2 --warmup 1 > $O/mehp_new.json 2> $O/mehp_new.err && \
FHE_LIB=fhe-sorting_amd/lib/ab_old.so timeout -k 10 300 python scripts/shard_rehearsal.py direct 8 > $O/shard_old.json 2> $O/shard_old.err && \
timeout -k 10 300 python scripts/shard_rehearsal.py direct 8 > $O/shard_new.json 2> $O/shard_new.err
