#!/bin/bash
# round 4: DPP row variants for the rescale (8) and key-switch-finish (16) rows on
# top of the new default (5 = inverse + HMult-tail rows): parity with every DPP
# row on (29), then bench A/B at the default 2 lanes
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r4k
mkdir -p $O
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
FHE_NTT_ROW_SHFL=29 timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_digests.py -k "not ring17 and not shipped" > $O/tests29.log 2>&1 || { echo "tests failed"; tail -40 $O/tests29.log; exit 1; }
tail -2 $O/tests29.log
run() {  # name shfl
  env FHE_NTT_ROW_SHFL=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --mask-steps 0 > $O/ab_$1.json 2> $O/ab_$1.err || { echo "bench $1 failed"; tail -5 $O/ab_$1.err; exit 1; }
  python - $O/ab_$1.json $1 <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']
ks = r['kernels_by_caller']
print(sys.argv[2], 'wall', d['ms_per_step'], 'clocked', r['clocked_ms_per_sort'], {k: v['avg_us'] for k, v in ks.items() if 'fwd' in k and ('rescale' in k or 'mul_tail' in k or 'ks_mod' in k)})
PY
}
run s5a 5 && run s13a 13 && run s21a 21 && run s29a 29 && run s5b 5 && run s13b 13 && run s21b 21 && run s29b 29 || exit 1
echo ALLOK
