#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench (with CPU baseline), rocprof kernel stats of the
# headline round (the roofline's region; --aes10-batch 0) and of the 10-round AES-128 run, and
# the PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs) of the NTT kernels on tools/ks_driver.
# Every GPU step has its own time limit; steps are chained so a failure stops the script.
# The per-dispatch kernel traces are deleted after each profile (the stats CSVs stay): with them
# the call's gpurun_out/ exceeded the 64 MiB that is merged back.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r01}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
 && echo "gpu tests ok" \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
 && echo "smoke ok" \
 && timeout -k 10 600 python bench.py --check ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
 && echo "bench ok" \
 && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o bench -- python bench.py --no-cpu-baseline --aes10-batch 0 ${BENCH_ARGS} > gpurun_out/prof_${TAG}.log 2>&1 \
 && rm -f gpurun_out/prof_${TAG}/*_kernel_trace.csv && echo "rocprof ok" \
 && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_aes10 -o aes10 -- python bench.py --no-cpu-baseline --steps 1 --warmup 0 ${BENCH_ARGS} > gpurun_out/prof_${TAG}_aes10.log 2>&1 \
 && rm -f gpurun_out/prof_${TAG}_aes10/*_kernel_trace.csv && echo "rocprof aes10 ok" \
 && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_fetch -o p -- ./tools/ks_driver 16 4 > gpurun_out/pmc_fetch.log 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_write -o p -- ./tools/ks_driver 16 4 > gpurun_out/pmc_write.log 2>&1 \
 && echo "pmc ok"
rc=$?
tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/smoke.log 2>/dev/null | tail -2; cat gpurun_out/bench_${TAG}.json 2>/dev/null
exit $rc
