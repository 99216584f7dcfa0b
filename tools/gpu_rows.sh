#!/bin/bash
# Row-layout dev loop on the GPU box: parity tests, stage split, bench (verified).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
B=${B:-4}
timeout -k 10 600 python -m pytest tests/test_aes_rows.py tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_rows.log 2>&1 && echo tests ok \
&& timeout -k 10 300 python tools/round_stages.py rows $B > gpurun_out/stages_rows.log 2>&1 && cat gpurun_out/stages_rows.log \
&& timeout -k 10 300 python bench.py --check --no-cpu-baseline --batch $B > gpurun_out/bench_rows.json 2>&1 && cat gpurun_out/bench_rows.json
rc=$?; tail -3 gpurun_out/pytest_rows.log; exit $rc
