#!/bin/bash
# A/B: adaptive target chunks in the basis conversions (FHE_CONV_CHUNK=64 = the
# old one-chunk launch) on configs 4 and 3, after the parity subset
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bootstrap.py -x -q --timeout 300 --timeout-method thread -k "modup or relinearised or rotations or batched or direct_sort_bit_exact or bootstrap_stages or bit_exact" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 0 64; do
  FHE_CONV_CHUNK=$v timeout -k 10 400 python bench.py --workload kway --steps 2 --no-cpu-baseline --no-roofline > $O/kway_$v.json 2> $O/kway_$v.err || { echo "kway $v failed"; tail -5 $O/kway_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/kway_$v.json'));print('kway chunk=$v', d['ms_per_step'], d['max_abs_err'])"
done
for v in 0 64; do
  FHE_CONV_CHUNK=$v timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-roofline > $O/direct_$v.json 2> $O/direct_$v.err || { echo "direct $v failed"; tail -5 $O/direct_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/direct_$v.json'));print('direct chunk=$v', d['ms_per_step'], d['max_abs_err'])"
done
echo ALLOK
