#!/bin/bash
# PMC passes over exactly one bench round step (--pmc-marks), each counter group in its own
# rocprofv3 run (--kernel-trace only): HBM bytes (FETCH_SIZE, WRITE_SIZE), fp64 instruction
# counts, SQ wave / wait cycles, L2 hit / miss; then the bootstrap kernel mix (gpu_r04_bootprof.sh).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-p4}
B1="bench.py --steps 1 --warmup 1 --pmc-marks --no-configs --aes10-batch 0 --no-cpu-baseline --client-batch 0 --no-harness --profile-steps 0 --no-check --config5 off"
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc_${n}_${TAG} -o p -- python3 $B1 > gpurun_out/pmc_${n}_${TAG}.json 2> gpurun_out/pmc_${n}_${TAG}.err \
    && rm -f gpurun_out/pmc_${n}_${TAG}/*kernel_trace.csv && echo "$n ok"
}
run fetch FETCH_SIZE \
 && run write WRITE_SIZE \
 && run f64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 \
 && run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SMEM \
 && run tcc TCC_HIT_sum TCC_MISS_sum \
 && if [ -z "$NOBOOT" ]; then TAG=${TAG}_boot bash tools/gpu_r04_bootprof.sh; fi
