#!/bin/bash
# A/B: MFMA linear sums with 2 column tiles per wave in 512-thread blocks
# (lib/ab_ls2.so) against the default 4 tiles / 256 threads; the MFMA parity
# tests and the digest tests on the A/B build first
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3ls2
mkdir -p $O
AB=fhe-sorting_amd/lib/ab_ls2.so
FHE_LIB=$AB timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_digests.py -x -q --timeout 200 --timeout-method thread > $O/tests_ab.log 2>&1 || { echo "ab tests failed"; tail -30 $O/tests_ab.log; exit 1; }
tail -2 $O/tests_ab.log
for V in def ab def2 ab2; do
  case $V in ab*) L=$AB;; *) L=;; esac
  FHE_LIB=$L timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline > $O/b_$V.json 2> $O/b_$V.err || { echo "bench $V failed"; tail -5 $O/b_$V.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_$V.json'));r=d['roofline'];print('$V', d['ms_per_step'], d['max_abs_err'], r['kernel'], r['frac'], {k:(v['avg_us'],v['share']) for k,v in list(r['kernels'].items())[:2]})"
done
echo ALLOK
