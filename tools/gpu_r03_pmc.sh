#!/bin/bash
# PMC passes over exactly one bench round step (--pmc-marks), each counter group in its own
# rocprofv3 run (--kernel-trace only), then the default bench.  Steps chained with &&.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-p}
B1="bench.py --steps 1 --warmup 1 --pmc-marks --no-configs --aes10-batch 0 --no-cpu-baseline --client-batch 0 --no-harness --profile-steps 0 --no-check ${PMC_ARGS}"
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_${TAG}.txt 2>&1; echo "counter list rc=$?"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_${TAG} -o p -- python3 $B1 > gpurun_out/pmc_fetch_${TAG}.json 2> gpurun_out/pmc_fetch_${TAG}.err \
 && echo "fetch ok" \
 && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_${TAG} -o p -- python3 $B1 > gpurun_out/pmc_write_${TAG}.json 2> gpurun_out/pmc_write_${TAG}.err \
 && echo "write ok" \
 && { timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 --kernel-trace --output-format csv -d gpurun_out/pmc_f64_${TAG} -o p -- python3 $B1 > gpurun_out/pmc_f64_${TAG}.json 2> gpurun_out/pmc_f64_${TAG}.err; echo "f64 rc=$?"; } \
 && rm -f gpurun_out/pmc_*_${TAG}/*kernel_trace.csv \
 && if [ -z "$NO_BENCH" ]; then timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err && echo "bench ok"; fi
rc=$?
grep -v "^W20\|^I20\|^E20" gpurun_out/bench_${TAG}.err 2>/dev/null | tail -3
exit $rc
