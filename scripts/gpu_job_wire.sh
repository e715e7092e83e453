#!/bin/bash
# wire format + CLI: GPU tests, then the reference CLI configuration end to end
# (N = 128, ring 2^16, CompositeSign(4, 3, 3), depth 42) through files in $TMPDIR
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wire.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/tests_wire.log 2>&1 || { echo "wire tests failed"; tail -40 gpurun_out/tests_wire.log; exit 1; }
tail -8 gpurun_out/tests_wire.log
N=${1:-128}
D=$(mktemp -d /tmp/fhecli.XXXX)
trap 'rm -rf "$D"' EXIT
t0=$(date +%s.%N)
timeout -k 10 300 python fhe-sorting_amd/client.py setup --dir $D --n $N --log-n 16 --scale-bits 50 --seed 3 > gpurun_out/cli_setup.log 2>&1 || { echo setup failed; cat gpurun_out/cli_setup.log; exit 1; }
t1=$(date +%s.%N)
timeout -k 10 120 python fhe-sorting_amd/client.py encrypt --dir $D --n $N --random 7 --output $D/x.bin || exit 1
t2=$(date +%s.%N)
for i in 1 2; do
  timeout -k 10 300 fhe-sorting_amd/bin/fhesort --cc $D/cc.bin --key_pub $D/key_pub.bin --key_mult $D/key_mult.bin --key_rot $D/key_rot.bin --input $D/x.bin --output $D/y.bin --n $N --timing 2>> gpurun_out/cli_timing.log || { echo cli failed; cat gpurun_out/cli_timing.log; exit 1; }
done
t3=$(date +%s.%N)
timeout -k 10 120 python fhe-sorting_amd/client.py decrypt --dir $D --n $N --input $D/y.bin --output $D/y.npy || exit 1
python - "$D" "$N" <<'PY' | tee gpurun_out/cli_n128.json
import json, os, sys
import numpy as np
d, N = sys.argv[1], int(sys.argv[2])
y = np.load(os.path.join(d, 'y.npy'))
v = np.random.default_rng(7).permutation(N) / N
sizes = {f: os.path.getsize(os.path.join(d, f)) for f in sorted(os.listdir(d)) if f.endswith('.bin')}
runs = [json.loads(l) for l in open('gpurun_out/cli_timing.log') if l.startswith('{')]
print(json.dumps({'N': N, 'max_abs_err': float(np.abs(y - np.sort(v)).max()), 'file_bytes': sizes, 'cli_runs': runs}))
PY
python -c "print('setup_s %.2f encrypt_s %.2f cli_2runs_s %.2f' % ($t1 - $t0, $t2 - $t1, $t3 - $t2))"
df -h /tmp | tail -1
echo ALLOK
