#!/bin/bash
# round 4: NTT parity with the 32-bit LDS exchange, A/B of the exchange width
# and of the forward DPP row pass, then the sort-only profile of the default build
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r4b
mkdir -p $O
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "ntt or relinearised or rotations or direct_sort_bit_exact or modup or rescale or ring_2_17" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for V in lds64 lds32 cwpe5 cwpe6; do
  FHE_LIB=$R/fhe-sorting_amd/lib/ab_$V.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > $O/ab_$V.json 2> $O/ab_$V.err || { echo "bench $V failed"; tail -5 $O/ab_$V.err; exit 1; }
done
FHE_NTT_ROW_SHFL=3 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > $O/ab_lds32_shfl3.json 2> $O/ab_lds32_shfl3.err || { echo "bench shfl3 failed"; tail -5 $O/ab_lds32_shfl3.err; exit 1; }
python - $O <<'PY'
import json, sys, os
for f in ('ab_lds64', 'ab_lds32', 'ab_cwpe5', 'ab_cwpe6', 'ab_lds32_shfl3'):
    d = json.load(open(os.path.join(sys.argv[1], f + '.json'))); r = d['roofline']
    print(f, d['ms_per_step'], r['clocked_ms_per_sort'])
    for k, v in r['kernels_by_caller'].items():
        print('   ', k, v)
PY
kill $TICK 2>/dev/null
bash scripts/gpu_job_r4prof.sh r4_base
