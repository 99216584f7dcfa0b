#!/bin/bash
# Memory-latency SQ counters (one pass each for the A = ab_old.so and B = in-tree builds) over one
# bench round step between marker kernels.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-sq2}
B1="bench.py --steps 1 --warmup 1 --pmc-marks --no-configs --aes10-batch 0 --no-cpu-baseline --client-batch 0 --no-harness --profile-steps 0 --no-check"
CNT="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAIT_ANY SQ_INSTS_VALU"
AESFHE_LIB=aes-fhe_amd/build/ab_old.so timeout -s KILL 240 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_A -o p -- python3 $B1 > gpurun_out/pmc_${TAG}_A.json 2> gpurun_out/pmc_${TAG}_A.err \
 && echo "A ok" \
 && timeout -s KILL 240 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_B -o p -- python3 $B1 > gpurun_out/pmc_${TAG}_B.json 2> gpurun_out/pmc_${TAG}_B.err \
 && echo "B ok" && rm -f gpurun_out/pmc_${TAG}_*/*kernel_trace.csv
