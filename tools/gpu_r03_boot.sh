#!/bin/bash
# bit-mode bootstrap (depth-optimal EvalMod + folded c_in): timing/phases, a step-by-step 10-round
# AES diagnosis, the GPU bootstrap / AES-128 tests and the bench's aes10 leg (GPU box)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-boot}
timeout -k 10 300 python -u tools/boot_bench.py --scale-bits 40 --special-primes 10 --batch ${PPC:-16} --phases > gpurun_out/${T}_boot.log 2>&1 || { tail -20 gpurun_out/${T}_boot.log; exit 1; }
cat gpurun_out/${T}_boot.log
timeout -k 10 300 python -u tools/aes10_diag.py 16 30 10 40 > gpurun_out/${T}_diag.log 2>&1 || { tail -20 gpurun_out/${T}_diag.log; exit 1; }
cat gpurun_out/${T}_diag.log
if [ -n "$DIAG17" ]; then
  timeout -k 10 400 python -u tools/aes10_diag.py 17 35 12 44 > gpurun_out/${T}_diag17.log 2>&1 || { tail -20 gpurun_out/${T}_diag17.log; exit 1; }
  cat gpurun_out/${T}_diag17.log
fi
timeout -k 10 600 python -u -m pytest ${PYTEST_FILES:-tests/test_bootstrap.py tests/test_aes128_full.py} -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/${T}_pytest.log
timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --no-configs --no-cpu-baseline --no-harness --client-batch 0 ${BENCH_ARGS} > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); a=d['aes128_10_rounds']
print('round', d['value'], d['ms_per_step']); print({k: a[k] for k in a if k not in ('pool',)})"
