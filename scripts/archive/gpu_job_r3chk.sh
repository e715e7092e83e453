#!/bin/bash
# adaptive block chunk of the MFMA linear sums: parity (MFMA tests, digests, PS
# series), then the headline and k-way bench lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3chk
mkdir -p $O
(while sleep 50; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_digests.py tests/test_gpu_parity.py tests/test_gpu_bootstrap.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('direct', d['ms_per_step'], d['max_abs_err'], r['kernel'], r['frac'], {k:(v['avg_us'],v['share']) for k,v in list(r['kernels'].items())[:2]})"
timeout -k 10 300 python bench.py --workload kway --steps 2 --no-cpu-baseline > $O/kway.json 2> $O/kway.err || { echo "kway failed"; tail -5 $O/kway.err; exit 1; }
python -c "import json;d=json.load(open('$O/kway.json'));r=d.get('roofline') or {};print('kway', d['ms_per_step'], r.get('kernel'), r.get('frac'))"
echo ALLOK
