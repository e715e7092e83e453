#!/bin/bash
# round 4: DPP (+ LDS row twiddles) for every forward row pass (FHE_NTT_ROW_SHFL
# 15 / 31) against the default 13, at the default two lanes; parity with 31 first
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r4n
mkdir -p $O
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
FHE_LIB=$R/fhe-sorting_amd/lib/_cm.so timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_rotate_members.py > $O/tests_cm.log 2>&1 || { echo "rotate_members tests failed"; tail -40 $O/tests_cm.log; exit 1; }
tail -1 $O/tests_cm.log
FHE_LIB=$R/fhe-sorting_amd/lib/_cm.so FHE_NTT_ROW_SHFL=31 timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_digests.py -k "not ring17 and not shipped" > $O/tests31.log 2>&1 || { echo "tests failed"; tail -40 $O/tests31.log; exit 1; }
tail -1 $O/tests31.log
run() {  # name shfl
  env FHE_LIB=$R/fhe-sorting_amd/lib/_cm.so FHE_NTT_ROW_SHFL=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --mask-steps 0 > $O/ab_$1.json 2> $O/ab_$1.err || { echo "bench $1 failed"; tail -5 $O/ab_$1.err; exit 1; }
  python - $O/ab_$1.json $1 <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']
ks = r['kernels_by_caller']
print(sys.argv[2], 'wall', d['ms_per_step'], 'clocked', r['clocked_ms_per_sort'], {k: v['avg_us'] for k, v in ks.items() if 'fwd' in k and ('modup' in k or 'ks_mod' in k) and 'true, 0' not in k})
PY
}
run s13a 13 && run s15a 15 && run s31a 31 && run s13b 13 && run s15b 15 && run s31b 31 || exit 1
echo ALLOK
