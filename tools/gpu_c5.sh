#!/bin/bash
# GPU session: GPU tests, then config 5's per-rank shard (N = 2^17, L = 35, 16 sets = 64
# reference ciphertexts' worth of blocks) with the 10-round run, then a rocprofv3 kernel summary
# of the config-5 round.  Each GPU step has its own limit; steps are chained with &&.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-c5}
C5="--log-n 17 --max-level 35 --special-primes 12 --scale-bits 44 --batch 16 --aes10-batch 16 --no-cpu-baseline"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1 \
 && echo "gpu tests ok" \
 && timeout -k 10 900 python bench.py $C5 --steps 2 --warmup 1 ${BENCH_ARGS} > gpurun_out/bench_c5_${TAG}.json 2> gpurun_out/bench_c5_${TAG}.err \
 && echo "config5 ok" \
 && if [ -n "$PROF" ]; then timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_${TAG} -o c5 -- python bench.py $C5 --steps 1 --warmup 1 --aes10-batch 0 --profile-steps 0 > gpurun_out/prof_c5_${TAG}.log 2>&1 && rm -f gpurun_out/prof_c5_${TAG}/*_kernel_trace.csv && echo "rocprof ok"; fi
rc=$?
tail -3 gpurun_out/pytest_gpu_${TAG}.log; cat gpurun_out/bench_c5_${TAG}.json 2>/dev/null; tail -3 gpurun_out/bench_c5_${TAG}.err 2>/dev/null
exit $rc
