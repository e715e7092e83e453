#!/bin/bash
# round 6 closing: the full GPU suite and smoke() on the final library, then the
# closing profile of the N=1024 sort (scripts/gpu_job_r4prof.sh); PART=side: the
# config-5 / config-4 profiles (profiles/pmc_*_mehp24.json, pmc_*_kway.json)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
T=${1:-r6_final}
O=gpurun_out/${T}_suite
mkdir -p $O
if [ "${PART:-main}" = main ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20; exit 1; }
  tail -3 $O/tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
  tail -3 $O/smoke.log
  bash scripts/gpu_job_r4prof.sh $T
else
  PMCSFX=_mehp24 bash scripts/gpu_job_r4prof.sh ${T}_mehp24 --workload mehp24 && \
  PMCSFX=_kway bash scripts/gpu_job_r4prof.sh ${T}_kway --workload kway
fi
