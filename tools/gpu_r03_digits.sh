#!/bin/bash
# Full GPU suite, then the round bench with the widest key-switch digits (default) against
# alpha = K, alternated.  Every step limited, chained with &&.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-dg}
ARGS="--no-configs --no-harness --aes10-batch 0 --no-cpu-baseline ${EXTRA}"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread ${PYTEST_K} > gpurun_out/pytest_${TAG}.log 2>&1 \
 && echo "gpu tests ok" \
 && timeout -k 10 400 python bench.py ${ARGS} > gpurun_out/bench_${TAG}_a1.json 2> gpurun_out/bench_${TAG}_a1.err \
 && echo "widest 1 ok" \
 && timeout -k 10 400 python bench.py --digit-primes 0 ${ARGS} > gpurun_out/bench_${TAG}_k1.json 2> gpurun_out/bench_${TAG}_k1.err \
 && echo "alpha=K ok" \
 && timeout -k 10 400 python bench.py ${ARGS} > gpurun_out/bench_${TAG}_a2.json 2> gpurun_out/bench_${TAG}_a2.err \
 && echo "widest 2 ok"
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_${TAG}.log | tail -8
for f in gpurun_out/bench_${TAG}_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print('$f', c['layout'], c.get('digit_primes'), c.get('dnum'), d['value'], d['ms_per_step'], c['verified'], (d.get('client_path') or {}).get('value'))" 2>/dev/null; done
exit $rc
