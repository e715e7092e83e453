#!/bin/bash
# round 5, closing profile of the benched library: the N=1024 sort (profiles/pmc_*.json)
# and configs 5 / 4 (profiles/pmc_*_mehp24.json, pmc_*_kway.json), each with its
# sort-only trace, FETCH / WRITE / SQ passes stamped with the library hash and the
# bench line that reads them
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
T=${1:-r5_final}
bash scripts/gpu_job_r4prof.sh $T && \
PMCSFX=_mehp24 bash scripts/gpu_job_r4prof.sh ${T}_mehp24 --workload mehp24 && \
PMCSFX=_kway bash scripts/gpu_job_r4prof.sh ${T}_kway --workload kway
