#!/bin/bash
# config 4 (k-way) and config 5 (MEHP24) on the MFMA build: the default mask
# (PS linear sums on MFMA) and, for MEHP24's wide digits (alpha 22, K 16), the
# ModUp / ModDown MFMA forms
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r3mfw
mkdir -p $O
(while sleep 50; do echo "tick $(date +%T)"; done) & TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -k 10 300 python bench.py --workload kway --steps 2 --no-cpu-baseline > $O/kway.json 2> $O/kway.err || { echo "kway failed"; tail -5 $O/kway.err; exit 1; }
python -c "import json;d=json.load(open('$O/kway.json'));r=d.get('roofline') or {};print('kway', d['ms_per_step'], d.get('bootstrap_ms'), r.get('kernel'), r.get('frac'))"
for V in 1 3 5; do
  FHE_MFMA=$V timeout -k 10 400 python bench.py --workload mehp24 --steps 1 --no-cpu-baseline --no-roofline > $O/mehp24_$V.json 2> $O/mehp24_$V.err || { echo "mehp24 $V failed"; tail -5 $O/mehp24_$V.err; exit 1; }
  python -c "import json;d=json.load(open('$O/mehp24_$V.json'));print('mehp24 mask $V', d['ms_per_step'], d.get('max_abs_err'))"
done
echo ALLOK
