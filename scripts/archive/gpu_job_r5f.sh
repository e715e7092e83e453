#!/bin/bash
# round 5: fused ModUp row pass + key-switch inner product (ntt_row_ks) --
# large-ring products and the digests, then the bench A/B (unfused / fused
# at 2 waves / fused at 3 waves with spills)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_f}
mkdir -p $O
FHE_KS_FUSE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "large_rings or batched or config2" --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
FHE_KS_FUSE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_digests.py -x -q --timeout 300 --timeout-method thread > $O/digests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_nofuse.json 2> $O/bench_nofuse.err && \
FHE_KS_FUSE=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_fuse.json 2> $O/bench_fuse.err && \
FHE_KS_FUSE=1 FHE_LIB=fhe-sorting_amd/lib/ab_kswpe3.so timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_fuse3.json 2> $O/bench_fuse3.err
[ -f $O/bench_fuse3.json ] && FHE_PS_XCD=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_psxcd0.json 2> $O/bench_psxcd0.err
# smaller stacks keep a lane's intermediates in the 256-MB infinity cache
for SL in "8 2" "16 2" "8 4" "4 2" "4 4"; do
  set -- $SL
  [ -f $O/bench_psxcd0.json ] && timeout -k 10 300 python bench.py --no-cpu-baseline --stack $1 --lanes $2 > $O/bench_stack$1_lanes$2.json 2> $O/bench_stack$1_lanes$2.err
done
true
