#!/bin/bash
# A/B of the linear-sum MFMA waves hint (default build vs lib/ab_lswpe0.so),
# then the headline profile flow (scripts/gpu_job_r3e.sh) on the default build
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3mfab
mkdir -p $O
for V in def ab def2; do
  if [ $V = ab ]; then L=fhe-sorting_amd/lib/ab_lswpe0.so; else L=; fi
  FHE_LIB=$L timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline > $O/b_$V.json 2> $O/b_$V.err || { echo "bench $V failed"; tail -5 $O/b_$V.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_$V.json'));r=d['roofline'];print('$V', d['ms_per_step'], r['kernel'], r['frac'], {k:(v['avg_us'],v['share']) for k,v in list(r['kernels'].items())[:3]})"
done
bash scripts/gpu_job_r3e.sh ${1:-r3_mf_final}
