#!/bin/bash
# A/B: coefficients per block of the MFMA linear sums (1024 default, 2048, 4096)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3ch
mkdir -p $O
for V in def ch2k ch4k def2 ch2k2 ch4k2; do
  case $V in ch2k*) L=fhe-sorting_amd/lib/ab_ch2k.so;; ch4k*) L=fhe-sorting_amd/lib/ab_ch4k.so;; *) L=;; esac
  FHE_LIB=$L timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline > $O/b_$V.json 2> $O/b_$V.err || { echo "bench $V failed"; tail -5 $O/b_$V.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_$V.json'));r=d['roofline'];print('$V', d['ms_per_step'], d['max_abs_err'], r['kernel'], r['frac'], {k:(v['avg_us'],v['share']) for k,v in list(r['kernels'].items())[:1]})"
done
echo ALLOK
