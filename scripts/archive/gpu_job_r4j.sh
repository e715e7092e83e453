#!/bin/bash
# round 4: leaf sums at 4 waves per SIMD (lib/_leaf.so: 128 VGPRs, the accumulate
# loads after the products) and the DPP HMult-tail row (FHE_NTT_ROW_SHFL=5), both
# at 2 lanes -- MFMA / digest parity on _leaf.so, then bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r4j
mkdir -p $O
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
FHE_LIB=$R/fhe-sorting_amd/lib/_leaf.so timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_mfma.py tests/test_gpu_digests.py -k "not ring17 and not shipped" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
run() {  # name lib-or-default [env]
  L=""; [ "$2" != default ] && L="FHE_LIB=$R/fhe-sorting_amd/lib/$2.so"
  env $L $3 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --mask-steps 0 --lanes 2 > $O/ab_$1.json 2> $O/ab_$1.err || { echo "bench $1 failed"; tail -5 $O/ab_$1.err; exit 1; }
  python - $O/ab_$1.json $1 <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']
ks = r['kernels']
print(sys.argv[2], 'wall', d['ms_per_step'], 'clocked', r['clocked_ms_per_sort'], {k: v['avg_us'] for k, v in ks.items() if 'leaf' in k or 'row' in k or ', 3,' in k})
PY
}
run def1 default && run leaf1 _leaf && run dpp1 default FHE_NTT_ROW_SHFL=5 && run leafdpp1 _leaf FHE_NTT_ROW_SHFL=5 && run def2 default && run leaf2 _leaf && run dpp2 default FHE_NTT_ROW_SHFL=5 && run leafdpp2 _leaf FHE_NTT_ROW_SHFL=5 || exit 1
echo ALLOK
