#!/bin/bash
# Round 6: counters of the fused conversion + column-pass kernel (bconv_cols.h) against the pair it
# replaced, cold caches (tools/modup_fused_bench <shape> 32 cold: the Infinity Cache flushed before
# each launch, as in the engine).  One rocprofv3 --pmc pass per counter group, summarised per
# kernel by tools/pmc_kernels.py.  SHAPE: 0 (ModUp digit 0) or -1 (ModDown).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-fpmc}
S=${SHAPE:-0}
B="./tools/modup_fused_bench $S 32 cold ${VAR:-1}"
timeout -k 10 120 $B > gpurun_out/${T}_time.log 2>&1 && cat gpurun_out/${T}_time.log \
 && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${T}_fetch -o p -- $B > /dev/null 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${T}_write -o p -- $B > /dev/null 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/${T}_sq -o p -- $B > /dev/null 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/${T}_tcc -o p -- $B > /dev/null 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d gpurun_out/${T}_sq2 -o p -- $B > /dev/null 2>&1 \
 && python3 tools/pmc_kernels.py gpurun_out/${T}_fetch gpurun_out/${T}_write gpurun_out/${T}_sq gpurun_out/${T}_tcc gpurun_out/${T}_sq2 > gpurun_out/${T}_pmc.txt \
 && rm -f gpurun_out/${T}_*/*kernel_trace.csv && cat gpurun_out/${T}_pmc.txt
