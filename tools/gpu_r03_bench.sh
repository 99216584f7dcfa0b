#!/bin/bash
# GPU tests selected by PYTEST_K (optional), then the default bench (BENCH_ARGS), each limited.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-b}
if [ -n "$PYTEST_FILES" ]; then
  timeout -k 10 600 python -u -m pytest $PYTEST_FILES -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
  echo "gpu tests ok"; tail -2 gpurun_out/pytest_${TAG}.log
fi
timeout -k 10 1000 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
rc=$?
tail -5 gpurun_out/bench_${TAG}.err
exit $rc
