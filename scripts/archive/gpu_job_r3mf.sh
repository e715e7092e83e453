#!/bin/bash
# MFMA sums of products: parity tests of the affected ops first (on a plain test
# failure, each kernel alone via the FHE_MFMA mask), then the digest + parity
# files, then the headline bench under FHE_MFMA = 7 (all), 1, 3 and 0 (VALU)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r3mf}
mkdir -p $O
(while sleep 50; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
SEL="chebyshev or sinc or linear_sum or modup or relinearised or rotations or wide_digits"
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py -x -v --timeout 120 --timeout-method thread > $O/tests_ps.log 2>&1
RC=$?
if [ $RC -ne 0 ]; then
  echo "ps tests failed rc=$RC"; grep -E 'PASSED|FAILED|Error|assert' $O/tests_ps.log | tail -30
  if [ $RC -eq 1 ]; then
    for M in 1 2 4; do
      FHE_MFMA=$M timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "$SEL" > $O/tests_ps_mask$M.log 2>&1
      R2=$?
      echo "mask $M rc=$R2"; tail -3 $O/tests_ps_mask$M.log
      [ $R2 -le 1 ] || exit 1
    done
  fi
  exit 1
fi
tail -3 $O/tests_ps.log
FHE_MFMA=7 timeout -k 10 400 python -u -m pytest tests/test_gpu_digests.py -x -q --timeout 200 --timeout-method thread > $O/tests_more.log 2>&1 || { echo "tests failed"; tail -40 $O/tests_more.log; exit 1; }
tail -3 $O/tests_more.log
for V in 1 0 7; do
  FHE_MFMA=$V timeout -k 10 300 python bench.py --steps 2 --no-cpu-baseline > $O/bench_mfma$V.json 2> $O/bench_mfma$V.err || { echo "bench $V failed"; tail -5 $O/bench_mfma$V.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_mfma$V.json'));r=d['roofline'];print('MFMA=$V', d['ms_per_step'], d.get('max_abs_err'), r['kernel'], r['frac'], {k:(v['avg_us'],v['GBps'],v['share']) for k,v in list(r['kernels'].items())[:8]})"
done
echo ALLOK
