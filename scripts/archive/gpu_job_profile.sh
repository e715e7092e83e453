#!/bin/bash
# Round profile: bench line, rocprofv3 kernel trace + stats of one sort, and
# two PMC passes (FETCH_SIZE, WRITE_SIZE) over every engine kernel.  The
# profiled runs use one lane, like bench.py's roofline pass, so per-launch
# durations and bytes match the live clock's.
# usage: [PMCOUT=pmc_traffic_mehp24.json] [PMC_EXCLUDE=regex] gpu_job_profile.sh TAG [extra bench args]
# (PMC_EXCLUDE: kernels left out of the counter passes -- the MEHP24 pass dies
#  inside the profiler's dispatch interception on k_permute at ring 2^17)
# (PMCOUT: the profiles/ file bench.py reads roofline.traffic from for this workload)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
TAG=${1:-run}; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline "$@" --lanes 1 > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
python scripts/trace_summary.py $O/trace/run_kernel_trace.csv > $O/trace_summary.txt && cat $O/trace_summary.txt || exit 1
gzip -f $O/trace/run_kernel_trace.csv
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 900 rocprofv3 --pmc $C --kernel-include-regex 'k_[a-z]' ${PMC_EXCLUDE:+--kernel-exclude-regex "$PMC_EXCLUDE"} --output-format csv -d "$R/$O/pmc_$C" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-roofline "$@" --lanes 1 > $O/pmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $O/pmc_$C.log; exit 1; }
done
python scripts/pmc_summary.py $O/pmc_FETCH_SIZE/run_counter_collection.csv $O/pmc_WRITE_SIZE/run_counter_collection.csv $O/pmc_traffic.json || exit 1
gzip -f $O/pmc_*/run_counter_collection.csv
cp $O/pmc_traffic.json profiles/${PMCOUT:-pmc_traffic.json}
timeout -k 10 900 python bench.py "$@" > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
echo ALLOK
