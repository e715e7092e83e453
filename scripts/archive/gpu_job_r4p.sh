#!/bin/bash
# round 4: plain sums with the segment-fastest grid
# ciphertexts (lib/_ps.so) -- parity incl. MEHP24 / k-way / bootstrap on that
# library, then bench A/B against the default
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r4p
mkdir -p $O
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
FHE_LIB=$R/fhe-sorting_amd/lib/_ps.so timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_mfma.py tests/test_gpu_mehp24.py tests/test_gpu_kway.py tests/test_gpu_bootstrap.py -k "not config4 and not 4096" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|passed|failed" $O/tests.log | tail -20; exit 1; }
tail -1 $O/tests.log
run() {  # name lib-or-default
  L=""; [ "$2" != default ] && L="FHE_LIB=$R/fhe-sorting_amd/lib/$2.so"
  env $L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --mask-steps 0 > $O/ab_$1.json 2> $O/ab_$1.err || { echo "bench $1 failed"; tail -5 $O/ab_$1.err; exit 1; }
  python - $O/ab_$1.json $1 <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']
ks = r['kernels']
print(sys.argv[2], 'wall', d['ms_per_step'], 'clocked', r['clocked_ms_per_sort'], {k: (v['launches'], v['avg_us']) for k, v in ks.items() if 'c0' in k or 'scalar' in k})
PY
}
run def1 default && run ps1 _ps && run def2 default && run ps2 _ps || exit 1
echo ALLOK
