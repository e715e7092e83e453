#!/bin/bash
# round 6 (verdict r5 item 3): the HBM ceiling -- scripts/row_pattern.hip with the
# guide's grid-stride 16-B copy, 100 launches per pattern, twice, with the GPU's
# clocks and power captured before, between and after
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r6_rates}
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/row_pattern.hip -o $O/row_pattern || exit 1
(amd-smi metric -c -p -t 2>&1 || rocm-smi --showclocks --showpower 2>&1) > $O/clocks_before.txt
( for i in 1 2 3 4 5 6 7 8; do amd-smi metric -c -p 2>&1 | grep -iE "GFX_0|SOCKET|CURRENT_SOCKET|MEM_0|CLK|POWER" | head -20; sleep 1; done ) > $O/clocks_during.txt &
SAMPLER=$!
timeout -k 10 300 $O/row_pattern > $O/row_pattern.jsonl || { kill $SAMPLER; exit 1; }
wait $SAMPLER
(amd-smi metric -c -p -t 2>&1 || rocm-smi --showclocks --showpower 2>&1) > $O/clocks_between.txt
timeout -k 10 300 $O/row_pattern > $O/row_pattern_2.jsonl || exit 1
(amd-smi metric -c -p -t 2>&1 || rocm-smi --showclocks --showpower 2>&1) > $O/clocks_after.txt
rm -f $O/row_pattern
cat $O/row_pattern.jsonl $O/row_pattern_2.jsonl
