#!/bin/bash
# Round-3 profiling session: rocprofv3 kernel summaries of the config-2 / config-3 legs, and the
# HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs, --kernel-trace only) of one bench
# round step on the current tree.  Each GPU step has its own limit; steps chained with &&.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r03a}
BENCH1="bench.py --steps 1 --warmup 1 --no-configs --aes10-batch 0 --no-cpu-baseline --profile-steps 0 --no-check"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c23_${TAG} -o c23 -- python3 tools/config_prof.py --legs ${LEGS:-2,3} > gpurun_out/c23_${TAG}.log 2>&1 \
 && echo "config legs profiled" \
 && rm -f gpurun_out/c23_${TAG}/*_kernel_trace.csv \
 && if [ -n "$PMC" ]; then \
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_${TAG} -o p -- python3 $BENCH1 > gpurun_out/pmc_fetch_${TAG}.log 2>&1 \
      && echo "fetch pass ok" \
      && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_${TAG} -o p -- python3 $BENCH1 > gpurun_out/pmc_write_${TAG}.log 2>&1 \
      && echo "write pass ok"; fi
rc=$?
tail -2 gpurun_out/c23_${TAG}.log
exit $rc
