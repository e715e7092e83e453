#!/bin/bash
# round 4: wide column NTT passes -- parity, then A/B against the round-3 passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r4c
mkdir -p $O
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "ntt or relinearised or rotations or direct_sort_bit_exact or modup or rescale or ring_2_17 or large_rings" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
FHE_LIB=$R/fhe-sorting_amd/lib/ab_wide8.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "ntt or relinearised or direct_sort_bit_exact" > $O/tests_wide8.log 2>&1 || { echo "tests wide8 failed"; tail -40 $O/tests_wide8.log; exit 1; }
tail -2 $O/tests_wide8.log
run() {  # name lib [env]
  env $3 FHE_LIB=$R/fhe-sorting_amd/lib/ab_$2.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 > $O/ab_$1.json 2> $O/ab_$1.err || { echo "bench $1 failed"; tail -5 $O/ab_$1.err; exit 1; }
  python - $O/ab_$1.json $1 <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']
ks = r['kernels_by_caller']
print(sys.argv[2], 'wall', d['ms_per_step'], 'clocked', r['clocked_ms_per_sort'],
      {k.split('@')[0].replace('k_ntt_', '') + '@' + k.split('@')[-1]: v['avg_us'] for k, v in ks.items() if 'ntt' in k})
PY
}
run base1 base && run wide4 wide4 && run wide8 wide8 && run widel64 widel64 && run base2 base && run wide8_shfl3 wide8 FHE_NTT_ROW_SHFL=3 && run wide8b wide8 && run wide4b wide4 || exit 1
echo ALLOK
