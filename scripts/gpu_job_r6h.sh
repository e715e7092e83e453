#!/bin/bash
# round 6: PS leaf sums with the column-pipelined group loop (FHE_LFF_PIPE=1,
# default build) against the old loop (lib/ab_lffpipe0.so): MFMA parity, digests,
# then the sort with its live clock, alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_h}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_digests.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20; exit 1; }
tail -2 $O/tests.log
for arm in pipe old pipe old; do
  case $arm in pipe) L="";; old) L="$R/fhe-sorting_amd/lib/ab_lffpipe0.so";; esac
  FHE_LIB=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$arm.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/bench_$arm.json')); k=d['roofline']['kernels']
print('$arm', d['ms_per_step'], d.get('max_abs_err'), {n: v['avg_us'] for n, v in k.items() if 'leaf' in n})"
done
