#!/bin/bash
# one-launch NTT dev check: correctness + timing variants + PMC passes (GPU box)
set -o pipefail
mkdir -p gpurun_out/nttq
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 5 120 ./tools/ntt_q_bench 468 > gpurun_out/nttq/time.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/nttq/pmc1 -o p -- ./tools/ntt_q_bench 468 > /dev/null 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/nttq/pmc2 -o p -- ./tools/ntt_q_bench 468 > /dev/null 2>&1 || exit 1
cat gpurun_out/nttq/time.log
