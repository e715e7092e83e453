#!/bin/bash
# round 5: SQ counters of the folded ModDown+rescale conversion against the VALU one
# (one sort each, one lane, the two conversion kernels only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/${1:-r5_x}
mkdir -p $O
export TMPDIR=/tmp
export ROC_AQL_QUEUE_SIZE=131072
B="--steps 1 --warmup 1 --no-cpu-baseline --no-roofline --lanes 1 --mask-steps 0"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_BUSY_CYCLES"
LDS="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE"
FHE_MODDOWN_FOLD=1 timeout -s KILL 300 rocprofv3 --pmc $SQ --kernel-include-regex 'k_moddown_rescale' --output-format csv -d "$R/$O/sq_fold" -o run -- python3 "$R/bench.py" $B > $O/sq_fold.log 2>&1 && \
FHE_MODDOWN_FOLD=1 timeout -s KILL 300 rocprofv3 --pmc $LDS --kernel-include-regex 'k_moddown_rescale' --output-format csv -d "$R/$O/lds_fold" -o run -- python3 "$R/bench.py" $B > $O/lds_fold.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc $SQ --kernel-include-regex 'k_moddown_rescale' --output-format csv -d "$R/$O/sq_valu" -o run -- python3 "$R/bench.py" $B > $O/sq_valu.log 2>&1 && \
FHE_MODDOWN_FOLD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex 'k_moddown_rescale' --output-format csv -d "$R/$O/trace_fold" -o run -- python3 "$R/bench.py" $B > $O/trace_fold.log 2>&1
