#!/bin/bash
# round 4: batched giant-step rotations in the index check (lib/_rot2.so) --
# DirectSort parity + digests on that library, then bench A/B against the default
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r4i
mkdir -p $O
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
export FHE_ROT_LIB=$R/fhe-sorting_amd/lib/_rot2.so
FHE_LIB=$FHE_ROT_LIB timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_digests.py -k "not ring17 and not shipped" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
run() {  # name lib-or-default
  L=""; [ "$2" != default ] && L="FHE_LIB=$R/fhe-sorting_amd/lib/$2.so"
  env $L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --mask-steps 0 > $O/ab_$1.json 2> $O/ab_$1.err || { echo "bench $1 failed"; tail -5 $O/ab_$1.err; exit 1; }
  python - $O/ab_$1.json $1 <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']
print(sys.argv[2], 'wall', d['ms_per_step'], 'clocked', r['clocked_ms_per_sort'], 'cold', d['cold_sort_s'], 'err', d['max_abs_err'])
PY
}
run rot2a _rot2 && run rot1a _rot && run def1 default && run rot2b _rot2 && run rot1b _rot || exit 1
echo ALLOK
