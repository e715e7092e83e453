#!/bin/bash
# round 5, second closing profile of the benched library (after the folded leaf
# sums, 32-leaf passes and the fused tensor): PART=main -- the N=1024 sort;
# PART=side -- configs 5 / 4 (profiles/pmc_*_mehp24.json, pmc_*_kway.json)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
T=${1:-r5_final2}
if [ "${PART:-main}" = main ]; then
  bash scripts/gpu_job_r4prof.sh $T
else
  PMCSFX=_mehp24 bash scripts/gpu_job_r4prof.sh ${T}_mehp24 --workload mehp24 && \
  PMCSFX=_kway bash scripts/gpu_job_r4prof.sh ${T}_kway --workload kway
fi
