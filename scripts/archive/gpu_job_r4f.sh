#!/bin/bash
# round 4: device encoder parity, a sort with per-sort masks, then the bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r4f
mkdir -p $O
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_encode.py tests/test_gpu_parity.py tests/test_gpu_digests.py -k "not ring17 and not shipped" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
run() {  # name lib-or-default [env]
  L=""; [ "$2" != default ] && L="FHE_LIB=$R/fhe-sorting_amd/lib/ab_$2.so"
  env $L $3 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 > $O/ab_$1.json 2> $O/ab_$1.err || { echo "bench $1 failed"; tail -5 $O/ab_$1.err; exit 1; }
  python - $O/ab_$1.json $1 <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']
ks = r['kernels_by_caller']
print(sys.argv[2], 'wall', d['ms_per_step'], 'clocked', r['clocked_ms_per_sort'], 'cold', d['cold_sort_s'],
      'per-sort masks', d['ms_per_step_masks_per_sort'], d['masks_per_sort_breakdown'],
      {k.split('@')[0].replace('k_ntt_', '') + '@' + k.split('@')[-1]: v['avg_us'] for k, v in ks.items() if 'row' in k})
PY
}
run all default && run norowtwl default FHE_NTT_TWL=0 && run nocoltwl nocoltwl && run rowwpe6 rwpe6 && run rowdpp_mt default FHE_NTT_ROW_SHFL=5 && run all2 default && run norowtwl2 default FHE_NTT_TWL=0 && run nocoltwl2 nocoltwl || exit 1
echo ALLOK
