#!/bin/bash
# PMC passes (each counter group in its own rocprofv3 run, --kernel-trace only; no sys/runtime
# traces): HBM-side bytes (FETCH_SIZE, WRITE_SIZE) of a one-step bench and of the NTT bench's
# copy kernel (calibration: its bytes are known), plus SQ stall counters of the bench.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
B=${B:-16}
run() {  # name, counters..., -- command
    local name=$1; shift
    timeout -k 10 600 rocprofv3 --pmc "$@" > gpurun_out/pmc_${name}.log 2>&1
}
run cal_fetch FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_cal_fetch -o p -- ./tools/ntt_bench \
&& run cal_write WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_cal_write -o p -- ./tools/ntt_bench \
&& run fetch FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o p -- ./tools/ks_driver $B 4 \
&& run write WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o p -- ./tools/ks_driver $B 4 \
&& run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o p -- ./tools/ks_driver $B 4
rc=$?
find gpurun_out/pmc_* -name "*counter_collection*" | head; du -sh gpurun_out/pmc_* 2>/dev/null | tail -6
exit $rc
