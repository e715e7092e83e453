#!/bin/bash
# round 6: config 4 (k-way, one-ciphertext ops) against the engine's launch-shape
# switches on the final library
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_n}
mkdir -p $O
for rep in 1 2; do
for arm in def full255 full117 shfl31 shfl15 chunk4 chunk8 mc4 auxon; do
  E="FHE_X=0"
  case $arm in full255) E="FHE_NTT_FULL=255";; full117) E="FHE_NTT_FULL=117";; shfl31) E="FHE_NTT_ROW_SHFL=31";; shfl15) E="FHE_NTT_ROW_SHFL=15";; chunk4) E="FHE_CONV_CHUNK=4";; chunk8) E="FHE_CONV_CHUNK=8";; mc4) E="FHE_KS_MC=4";; auxon) E="FHE_NTT_AUX=1";; esac
  env $E timeout -k 10 200 python bench.py --workload kway --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/kway_${arm}_$rep.json 2>> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json; d=json.load(open('$O/kway_${arm}_$rep.json')); print('$arm', $rep, d['ms_per_step'], d.get('max_abs_err'))"
done
done
