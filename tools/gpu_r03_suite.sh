#!/bin/bash
# GPU test suite + the config legs (timed, FIPS-verified).  Steps chained with &&, each limited.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-suite}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread ${PYTEST_K} > gpurun_out/pytest_${TAG}.log 2>&1 \
 && echo "gpu tests ok" \
 && timeout -k 10 300 python3 tools/config_prof.py --legs ${LEGS:-2,3} --reps 2 > gpurun_out/legs_${TAG}.json 2> gpurun_out/legs_${TAG}.err \
 && echo "legs ok"
rc=$?
tail -4 gpurun_out/pytest_${TAG}.log; cat gpurun_out/legs_${TAG}.json 2>/dev/null
exit $rc
