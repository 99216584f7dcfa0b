#!/bin/bash
# PMC passes over tools/ks_driver (one counter group per run): HBM bytes, L2 hits, SQ issue split
set -o pipefail
mkdir -p gpurun_out/pmcks
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { local n=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmcks/$n -o p -- ./tools/ks_driver 16 4 > gpurun_out/pmcks/$n.log 2>&1; }
run fetch FETCH_SIZE && run write WRITE_SIZE && run tcc TCC_HIT_sum TCC_MISS_sum \
 && run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_LDS
