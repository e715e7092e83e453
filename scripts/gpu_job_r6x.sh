#!/bin/bash
# round 6 A/B: the folded leaf sums' six-digit rows for the FP primes (FHE_LEAF_SIX=1,
# default; 0 = the eight-digit rows): parity (MFMA, HMult parity, digests, MEHP24),
# then the N=1024 sort and MEHP24 alternated, with the live clock's leaf-sum times
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_x}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_mehp24.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR|passed|failed|Error" $O/tests.log | tail -20; exit 1; }
tail -2 $O/tests.log
for v in 0 1 0 1 0 1; do
  FHE_LEAF_SIX=$v timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_$v.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_$v.json')); print('sort six=$v', d['ms_per_step'], d.get('max_abs_err'))" | tee -a $O/ab.txt
done
for v in 0 1; do
  FHE_LEAF_SIX=$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/roof_$v.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/roof_$v.json')); r=d['roofline']
for k,v in sorted(r['kernels'].items()):
    if 'leaf' in k: print('six=$v', k, json.dumps(v)[:200])
" | tee -a $O/ab.txt
done
for v in 0 1; do
  FHE_LEAF_SIX=$v timeout -k 10 240 python bench.py --workload mehp24 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/mehp24.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/mehp24.json')); print('mehp24 six=$v', d['ms_per_step'], d.get('max_abs_err'))" | tee -a $O/ab.txt
done
