#!/bin/bash
# round 4: 32-bit LDS exchanges in the column passes again, now that the column
# twiddles sit in LDS and the inverse column pass needs only 72 VGPRs (7 waves
# per SIMD once the tile is 21.5 KB); with and without a 5-wave VGPR cap on the
# forward column passes.  Parity on the capped build, then bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r4l
mkdir -p $O
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
for V in lds32w5 lds32; do
FHE_LIB=$R/fhe-sorting_amd/lib/ab_$V.so timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_digests.py -k "not ring17 and not shipped" > $O/tests_$V.log 2>&1 || { echo "tests $V failed"; tail -40 $O/tests_$V.log; exit 1; }
tail -1 $O/tests_$V.log
done
run() {  # name lib-or-default
  L=""; [ "$2" != default ] && L="FHE_LIB=$R/fhe-sorting_amd/lib/ab_$2.so"
  env $L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --mask-steps 0 > $O/ab_$1.json 2> $O/ab_$1.err || { echo "bench $1 failed"; tail -5 $O/ab_$1.err; exit 1; }
  python - $O/ab_$1.json $1 <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']
ks = r['kernels']
print(sys.argv[2], 'wall', d['ms_per_step'], 'clocked', r['clocked_ms_per_sort'], {k: v['avg_us'] for k, v in ks.items() if ', true, ' in k or 'inv<' in k})
PY
}
run def1 default && run l1 lds32 && run w1 lds32w5 && run def2 default && run l2 lds32 && run w2 lds32w5 || exit 1
echo ALLOK
