#!/bin/bash
# round 4, closing call on the final library: the whole GPU suite, smoke(), then
# the closing profiles of all three workloads (scripts/gpu_job_r4final.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
T=${1:-r4_final4}
bash scripts/gpu_job_r4suite.sh ${T}_suite && bash scripts/gpu_job_r4final.sh $T
