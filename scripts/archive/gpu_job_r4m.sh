#!/bin/bash
# round 4: buffer-addressed column passes + scalar column twiddles (default
# build, with 32-bit column exchanges) vs the same without them -- parity on
# the default build incl. ring 2^17 (512-point columns) and MEHP24, then A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r4m
mkdir -p $O
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_mfma.py tests/test_gpu_mehp24.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|passed|failed" $O/tests.log | tail -20; exit 1; }
tail -1 $O/tests.log
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
run def1 default && run nobuf1 nobuf && run noscal1 noscal && run def2 default && run nobuf2 nobuf && run noscal2 noscal || exit 1
echo ALLOK
