#!/bin/bash
# Counters per kernel of the bit bootstrap (tools/boot_bench.py at the bench's parameters, 64 bit
# ciphertexts per call, 5-map CtS): HBM bytes (FETCH_SIZE, WRITE_SIZE), SQ wave / wait / issue
# cycles, L2 hit / miss -- each group in its own rocprofv3 --pmc pass with the kernel trace --
# summarised per kernel by tools/pmc_kernels.py.  BENCH_ARGS overrides the workload.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-bpmc5}
BB=${BENCH_ARGS:-"tools/boot_bench.py --scale-bits 40 --special-primes 10 --digit-primes 12 --batch 32 --reps 1 --cts-groups 5"}
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/${TAG}_$n -o p -- python3 $BB > gpurun_out/${TAG}_$n.log 2>&1 && echo "$n ok"
}
run fetch FETCH_SIZE \
 && run write WRITE_SIZE \
 && run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SMEM \
 && run tcc TCC_HIT_sum TCC_MISS_sum \
 && python3 tools/pmc_kernels.py gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write gpurun_out/${TAG}_sq gpurun_out/${TAG}_tcc > gpurun_out/${TAG}_summary.txt \
 && rm -f gpurun_out/${TAG}_*/*kernel_trace.csv \
 && head -40 gpurun_out/${TAG}_summary.txt
