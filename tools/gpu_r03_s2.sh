#!/bin/bash
# GPU suite, config legs + reference harness (timed, verified), one SQ-counter PMC pass over a
# bench round step.  Steps chained with &&, each limited.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-s2}
B1="bench.py --steps 1 --warmup 1 --pmc-marks --no-configs --aes10-batch 0 --no-cpu-baseline --client-batch 0 --no-harness --profile-steps 0 --no-check"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread ${PYTEST_K} > gpurun_out/pytest_${TAG}.log 2>&1 \
 && echo "gpu tests ok" && tail -1 gpurun_out/pytest_${TAG}.log \
 && timeout -k 10 300 python3 -u tools/config_prof.py --legs 2,3,h > gpurun_out/legs_${TAG}.json 2> gpurun_out/legs_${TAG}.err \
 && echo "legs ok" \
 && if [ -n "$SQ" ]; then timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SMEM --kernel-trace --output-format csv -d gpurun_out/pmc_sq_${TAG} -o p -- python3 $B1 > gpurun_out/pmc_sq_${TAG}.json 2> gpurun_out/pmc_sq_${TAG}.err && echo "sq ok"; fi
rc=$?
tail -4 gpurun_out/pytest_${TAG}.log; cat gpurun_out/legs_${TAG}.json 2>/dev/null
exit $rc
