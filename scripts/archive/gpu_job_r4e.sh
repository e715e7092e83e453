#!/bin/bash
# round 4: one-pass leaf sums (k_leaf_sums_mfma) + pipelined forward column
# passes -- parity (incl. the full-size digests), then A/B of the column pipe
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r4e
mkdir -p $O
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_gpu_mfma.py tests/test_gpu_parity.py -k "not ring17 and not shipped" tests/test_gpu_digests.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
run() {  # name lib [env]
  env $3 FHE_LIB=$R/fhe-sorting_amd/lib/ab_$2.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 > $O/ab_$1.json 2> $O/ab_$1.err || { echo "bench $1 failed"; tail -5 $O/ab_$1.err; exit 1; }
  python - $O/ab_$1.json $1 <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']
ks = r['kernels_by_caller']
print(sys.argv[2], 'wall', d['ms_per_step'], 'clocked', r['clocked_ms_per_sort'], 'err', d['max_abs_err'],
      'leaf family', {k: v for k, v in r['families'].items() if 'leaf' in k or 'linear' in k},
      {k.split('@')[0].replace('k_ntt_', '') + '@' + k.split('@')[-1]: v['avg_us'] for k, v in ks.items() if 'ntt' in k})
PY
}
run nopipe1 nopipe && run pipe1 pipe && run nopipe2 nopipe && run pipe2 pipe || exit 1
echo ALLOK
