#!/bin/bash
# One-launch forward NTT record: tools/ntt_q_bench.hip's timings (two-pass,
# the quarter-transform kernels k_nttf_fwd_q / _q2, their memory-skeleton modes, copies), then its
# kernels' counters -- HBM bytes, SQ wait / issue, L2 hits -- one rocprofv3 --pmc pass per group
# with the kernel trace, summarised per kernel by tools/pmc_kernels.py.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-nttq}
timeout -k 10 120 ./tools/ntt_q_bench > gpurun_out/${T}_time.log 2>&1 && cat gpurun_out/${T}_time.log \
 && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${T}_fetch -o p -- ./tools/ntt_q_bench > /dev/null 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${T}_write -o p -- ./tools/ntt_q_bench > /dev/null 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/${T}_sq -o p -- ./tools/ntt_q_bench > /dev/null 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/${T}_tcc -o p -- ./tools/ntt_q_bench > /dev/null 2>&1 \
 && python3 tools/pmc_kernels.py gpurun_out/${T}_fetch gpurun_out/${T}_write gpurun_out/${T}_sq gpurun_out/${T}_tcc > gpurun_out/${T}_pmc.txt \
 && rm -f gpurun_out/${T}_*/*kernel_trace.csv && cat gpurun_out/${T}_pmc.txt
