#!/bin/bash
# round 6 (verdict r5 item 2): the integer-class relinearisation targets through the
# fused row-pass + inner-product kernel too (FHE_KS_FUSE_INT=1) -- parity, then
# the sort with its live clock and phases, alternating with the default
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_i}
mkdir -p $O
FHE_KS_FUSE_INT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py -x -q --timeout 300 --timeout-method thread -k "large_rings or config or digest" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20; exit 1; }
tail -2 $O/tests.log
for arm in int1 def int1 def; do
  case $arm in int1) E="FHE_KS_FUSE_INT=1";; def) E="FHE_KS_FUSE_INT=0";; esac
  env $E timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$arm.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/bench_$arm.json')); r=d['roofline']; k=r['kernels']
print('$arm', d['ms_per_step'], d.get('max_abs_err'), 'rank', r['phases']['rank_batches']['ms'], r['phases']['rank_batches']['kernel_over_op_bytes'], 'index', r['phases']['index_batches']['ms'])
print('   ', {n: (v['avg_us'], v.get('launches')) for n, v in k.items() if 'row_ks' in n or 'ks_inner' in n or 'fwd_row<0' in n})"
done
