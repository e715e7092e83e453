#!/bin/bash
# round 5: A/B of the FULL-grid mask with the FP passes (headline) and of the
# MFMA conversions at MEHP24's K = 16 / alpha = 22
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_e}
mkdir -p $O
for FM in 181 189 245 253; do
  FHE_NTT_FULL=$FM timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_full$FM.json 2> $O/bench_full$FM.err || exit 1
done
for MF in 1 3 5; do
  FHE_MFMA=$MF timeout -k 10 400 python bench.py --workload mehp24 --no-cpu-baseline > $O/mehp_mf$MF.json 2> $O/mehp_mf$MF.err || exit 1
done
