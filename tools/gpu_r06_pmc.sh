#!/bin/bash
# PMC passes over exactly one bench round step (--pmc-marks), each counter group in its own
# rocprofv3 run (--kernel-trace only): HBM bytes (FETCH_SIZE, WRITE_SIZE), fp64 instruction counts,
# SQ wave / wait cycles, L2 hit / miss.  Locally afterwards: tools/pmc_traffic.py (the record
# bench.py reads, profiles/r06/pmc/round_traffic.json) and tools/pmc_kernels.py (per kernel).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-p6}
B1="bench.py --steps 1 --warmup 1 --pmc-marks --no-configs --aes10-batch 0 --no-cpu-baseline --client-batch 0 --no-harness --profile-steps 0 --no-check --config5 off"
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc_${n}_${T} -o p -- python3 $B1 > gpurun_out/pmc_${n}_${T}.json 2> gpurun_out/pmc_${n}_${T}.err && echo "$n ok"
}
run fetch FETCH_SIZE \
 && run write WRITE_SIZE \
 && run f64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 \
 && run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SMEM \
 && run tcc TCC_HIT_sum TCC_MISS_sum \
 && du -sh gpurun_out/pmc_*_${T}
