#!/bin/bash
# Sliced layout (columns as batch elements, ShiftRows a batch permutation) against the rows
# layout (ShiftRows by rotations): GPU tests of both, then the round bench alternated
# sliced / rows / sliced on one box.  Every step limited, chained with &&.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-sl}
ARGS="--no-configs --no-harness --aes10-batch 0 --no-cpu-baseline ${EXTRA}"
timeout -k 10 600 python -u -m pytest tests/test_aes_rows.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 \
 && echo "gpu tests ok" && tail -2 gpurun_out/pytest_${TAG}.log \
 && timeout -k 10 400 python bench.py --layout sliced ${ARGS} > gpurun_out/bench_${TAG}_s1.json 2> gpurun_out/bench_${TAG}_s1.err \
 && echo "sliced 1 ok" \
 && timeout -k 10 400 python bench.py --layout rows ${ARGS} > gpurun_out/bench_${TAG}_r1.json 2> gpurun_out/bench_${TAG}_r1.err \
 && echo "rows 1 ok" \
 && timeout -k 10 400 python bench.py --layout sliced ${ARGS} > gpurun_out/bench_${TAG}_s2.json 2> gpurun_out/bench_${TAG}_s2.err \
 && echo "sliced 2 ok"
rc=$?
tail -30 gpurun_out/pytest_${TAG}.log | grep -E "passed|failed|Error" ; for f in gpurun_out/bench_${TAG}_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['config']['layout'], d['value'], d['ms_per_step'], d['config']['verified'], (d.get('client_path') or {}).get('value'))" 2>/dev/null; done
exit $rc
