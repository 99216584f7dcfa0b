#!/bin/bash
# Round-2 GPU session: GPU tests, smoke, default bench (FIPS-checked), rocprof kernel stats of
# the headline round.  Every GPU step has its own time limit; steps are chained with &&.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r02}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1 \
 && echo "gpu tests ok" \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 \
 && echo "smoke ok" \
 && timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
 && echo "bench ok"
rc=$?
tail -5 gpurun_out/pytest_gpu_${TAG}.log; tail -2 gpurun_out/smoke_${TAG}.log 2>/dev/null; cat gpurun_out/bench_${TAG}.json 2>/dev/null; tail -5 gpurun_out/bench_${TAG}.err 2>/dev/null
exit $rc
