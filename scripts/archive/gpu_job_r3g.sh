#!/bin/bash
# round 3: MEHP24 (config 5) PMC passes restricted to its dominant kernel (the
# ring-2^17 ModUp column pass): with every kernel counted, the pass serialises
# ~45k dispatches and did not finish in 500 s (r3d); FETCH_SIZE, WRITE_SIZE and
# SQ, fault report on
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3g
mkdir -p $O
# librocprofiler-sdk reads AQL packets past the end of the 16384-packet (1 MiB)
# queue ring when the write index wraps (r3g: faulting `cmpb $2, (%rax)` at
# librocprofiler-sdk.so.1.1.0+0x1e72fb on the first byte after a 1 MiB ring); a
# 131072-packet ring never wraps within this run
export TMPDIR=/tmp FHE_FAULT_REPORT=1 ROC_AQL_QUEUE_SIZE=131072
(while sleep 50; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
RX='k_ntt_fwd<9, 5, true|k_ntt_inv<9, 5, true|k_modup_convert|k_tensor|k_ks_inner'
B="--workload mehp24 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --lanes 1"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 420 rocprofv3 --pmc $C --kernel-include-regex "$RX" --output-format csv -d "$R/$O/pmc_$C" -o run -- python3 "$R/bench.py" $B > $O/pmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; grep -A8 "fhe fault report\] SIG" $O/pmc_$C.log | head -20
  [ $rc -eq 0 ] || { tail -5 $O/pmc_$C.log; exit 1; }
done
timeout -s KILL 420 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$RX" --output-format csv -d "$R/$O/pmc_SQ" -o run -- python3 "$R/bench.py" $B > $O/pmc_SQ.log 2>&1 || { echo "pmc SQ failed"; tail -5 $O/pmc_SQ.log; exit 1; }
python scripts/pmc_summary.py $O/pmc_FETCH_SIZE/run_counter_collection.csv $O/pmc_WRITE_SIZE/run_counter_collection.csv $O/pmc_traffic_mehp24.json > $O/pmc_traffic_mehp24.txt || exit 1
python scripts/pmc_sq_summary.py $O/pmc_SQ/run_counter_collection.csv $O/pmc_sq_mehp24.json > $O/pmc_sq_mehp24.txt || exit 1
gzip -f $O/pmc_*/run_counter_collection.csv
cp $O/pmc_traffic_mehp24.json $O/pmc_sq_mehp24.json profiles/
cat $O/pmc_traffic_mehp24.txt $O/pmc_sq_mehp24.txt
timeout -k 10 500 python bench.py --workload mehp24 --steps 1 --no-cpu-baseline > $O/bench_mehp24.json 2> $O/bench_mehp24.err || { echo "bench failed"; tail -5 $O/bench_mehp24.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_mehp24.json'));r=d['roofline'];print(d['ms_per_step'], r['kernel'], r['frac'], r.get('traffic'), r.get('valu_frac'))"
echo ALLOK
