#!/bin/bash
# GPU session: GPU tests, the default bench, config 5's shard with its 10-round run, then the
# single-launch NTT experiment (tools/ntt_fuse_bench).  Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-ar}
C5="--log-n 17 --max-level 35 --special-primes 12 --scale-bits 44 --batch 16 --aes10-batch 16 --no-cpu-baseline"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1 \
 && echo "gpu tests ok" \
 && timeout -k 10 900 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
 && echo "bench ok" \
 && timeout -k 10 900 python bench.py $C5 --steps 2 --warmup 1 --no-configs > gpurun_out/bench_c5_${TAG}.json 2> gpurun_out/bench_c5_${TAG}.err \
 && echo "config5 ok" \
 && if [ -x tools/ntt_fuse_bench ]; then timeout -k 10 120 ./tools/ntt_fuse_bench > gpurun_out/ntt_fuse_${TAG}.log 2>&1; echo "fuse rc $?"; cat gpurun_out/ntt_fuse_${TAG}.log; fi
rc=$?
tail -3 gpurun_out/pytest_gpu_${TAG}.log; cat gpurun_out/bench_${TAG}.json gpurun_out/bench_c5_${TAG}.json 2>/dev/null | cut -c1-400
exit $rc
