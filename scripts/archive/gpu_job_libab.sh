#!/bin/bash
# A/B of build variants (scripts/build_ab.sh): gpu_job_libab.sh name1 name2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out
i=0
for V in "$@"; do
  i=$((i+1))
  FHE_LIB=$R/fhe-sorting_amd/lib/ab_$V.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/libab_${i}_$V.json 2>gpurun_out/libab_${i}_$V.err || { echo "bench $V failed"; tail -5 gpurun_out/libab_${i}_$V.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/libab_${i}_$V.json'));r=d['roofline'];print('$V', d['ms_per_step'], r['clocked_ms_per_sort'], {k:v['avg_us'] for k,v in list(r['kernels_by_caller'].items())[:9]})"
done
echo ALLOK
