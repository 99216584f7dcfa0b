#!/bin/bash
# Closing GPU session: the whole -m gpu suite, smoke(), the default bench, then config 5's shard.
# Steps chained with &&, each limited.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-close}
C5="--log-n 17 --max-level 35 --special-primes 12 --scale-bits 44 --batch 16 --aes10-batch 16 --no-cpu-baseline --no-configs --no-harness --client-batch 0"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 \
 && echo "gpu tests ok" && tail -1 gpurun_out/pytest_${TAG}.log \
 && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_${TAG}.log 2>&1 \
 && tail -1 gpurun_out/smoke_${TAG}.log \
 && timeout -k 10 900 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
 && echo "bench ok" \
 && timeout -k 10 900 python -u bench.py $C5 --steps 2 --warmup 1 > gpurun_out/bench_c5_${TAG}.json 2> gpurun_out/bench_c5_${TAG}.err \
 && echo "config5 ok"
rc=$?
tail -3 gpurun_out/pytest_${TAG}.log
exit $rc
