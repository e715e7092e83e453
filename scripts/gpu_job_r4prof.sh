#!/bin/bash
# Round-4 profile of exactly the benched build, the sort only:
#   1. rocprofv3 kernel trace + stats of one timed sort (FHE_PROF_REGION=1:
#      marker kernels bracket the timed sort and the summaries keep only the
#      dispatches between them -- key generation, encryption and the warmup sort
#      are left out), one lane like bench.py's live clock;
#   2. FETCH_SIZE, WRITE_SIZE and SQ PMC passes over the same region;
#   3. the tables stamped with the libfhesort.so SHA-256 (scripts/pmc_meta.py),
#      copied into profiles/ of this box so the closing bench line reads them;
#   4. the default bench line.
# usage: gpu_job_r4prof.sh TAG [extra bench args]   (PMCSFX=_mehp24 / _kway for the side workloads)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
TAG=${1:-r4prof}; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
export FHE_PROF_REGION=1
# an 8 MiB AQL ring: the profiler's dispatch interception faults when HIP's
# default 16,384-packet ring wraps under a --pmc pass (the
# device mask encoder's launches made the N=1024 sort wrap it too)
export ROC_AQL_QUEUE_SIZE=131072
(while sleep 60; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
B="--steps 1 --warmup 1 --no-cpu-baseline --no-roofline --lanes 1 --mask-steps 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o run -- python3 "$R/bench.py" $B "$@" > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
python scripts/trace_summary.py $O/trace/run_kernel_trace.csv --stats-out $O/region_kernel_stats.csv > $O/trace_summary.txt && head -40 $O/trace_summary.txt || exit 1
cp $O/trace/run_kernel_stats.csv $O/run_kernel_stats.csv
gzip -f $O/trace/run_kernel_trace.csv
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 600 rocprofv3 --pmc $C --kernel-include-regex 'k_[a-z]' --output-format csv -d "$R/$O/pmc_$C" -o run -- python3 "$R/bench.py" $B "$@" > $O/pmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $O/pmc_$C.log; exit 1; }
done
timeout -s KILL 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_BUSY_CYCLES --kernel-include-regex 'k_[a-z]' --output-format csv -d "$R/$O/pmc_sq" -o run -- python3 "$R/bench.py" $B "$@" > $O/pmc_sq.log 2>&1 || { echo "pmc sq failed"; tail -5 $O/pmc_sq.log; exit 1; }
export FHE_PMC_NOTE="sort only (dispatches between the k_region_begin / k_region_end markers around the timed sort), one lane, bench.py $B $*"
python scripts/pmc_summary.py $O/pmc_FETCH_SIZE/run_counter_collection.csv $O/pmc_WRITE_SIZE/run_counter_collection.csv $O/pmc_traffic${PMCSFX}.json > $O/pmc_traffic.txt || exit 1
python scripts/pmc_sq_summary.py $O/pmc_sq/run_counter_collection.csv $O/pmc_sq${PMCSFX}.json > $O/pmc_sq.txt || exit 1
gzip -f $O/pmc_*/run_counter_collection.csv
cp $O/pmc_traffic${PMCSFX}.json $O/pmc_sq${PMCSFX}.json profiles/
unset FHE_PROF_REGION ROC_AQL_QUEUE_SIZE
timeout -k 10 600 python bench.py "$@" > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python - "$O/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline'] or {}
print(d['ms_per_step'], d['value'], d.get('max_abs_err'))
for k in ('kernel', 'frac', 'traffic_ratio', 'valu_frac', 'mfma_frac', 'limiter', 'avg_us'):
    print(' ', k, r.get(k))
f = r.get('by_family', {})
print('  family', f.get('kernel'), f.get('frac'), f.get('traffic_ratio'), f.get('valu_frac'), f.get('limiter'))
print('  pmc', r.get('pmc_source'))
PY
echo ALLOK
