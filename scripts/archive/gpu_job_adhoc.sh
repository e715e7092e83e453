set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_adhoc.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/tests_adhoc.log; exit 1; }
tail -1 gpurun_out/tests_adhoc.log
for V in 0 1 3 5 0 1; do
FHE_NTT_ROW_SHFL=$V timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 > gpurun_out/bench_v$V.json 2>gpurun_out/bench_v$V.err || { echo "bench $V failed"; tail -5 gpurun_out/bench_v$V.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_v$V.json'));r=d['roofline'];print('V$V', d['ms_per_step'], r['kernel'], r['frac'], {k:(v['avg_us'],v['GBps']) for k,v in list(r['kernels'].items())[:8]})"
done
