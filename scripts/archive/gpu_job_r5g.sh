#!/bin/bash
# round 5: hybrid fused relinearisation (FP targets fused, integer targets
# row pass + ks_inner) -- the whole GPU suite, then the bench A/B and config 5
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_g}
mkdir -p $O
FHE_KS_FUSE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "large_rings or batched" --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
FHE_KS_FUSE=1 timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 && \
FHE_KS_FUSE=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_nofuse.json 2> $O/bench_nofuse.err && \
FHE_KS_FUSE=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_fuse.json 2> $O/bench_fuse.err && \
FHE_KS_FUSE=1 timeout -k 10 400 python bench.py --workload mehp24 --no-cpu-baseline > $O/mehp24.json 2> $O/mehp24.err
