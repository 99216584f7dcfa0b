#!/bin/bash
# Round-2 GPU session: GPU tests, smoke, default bench (FIPS-checked), optional config-5 bench
# leg.  Every GPU step has its own time limit; steps are chained with &&.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r02}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1 \
 && echo "gpu tests ok" \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 \
 && echo "smoke ok" \
 && timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
 && echo "bench ok" \
 && if [ -n "$CONFIG5" ]; then timeout -k 10 900 python bench.py --log-n 17 --max-level 35 --special-primes 12 --scale-bits 44 --batch 16 --aes10-batch 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5_${TAG}.json 2> gpurun_out/bench_c5_${TAG}.err && echo "config5 ok"; fi
rc=$?
tail -5 gpurun_out/pytest_gpu_${TAG}.log; tail -2 gpurun_out/smoke_${TAG}.log 2>/dev/null; cat gpurun_out/bench_${TAG}.json 2>/dev/null; tail -5 gpurun_out/bench_${TAG}.err 2>/dev/null; cat gpurun_out/bench_c5_${TAG}.json 2>/dev/null; tail -3 gpurun_out/bench_c5_${TAG}.err 2>/dev/null
exit $rc
