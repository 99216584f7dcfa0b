#!/bin/bash
# Round 5 A/B on one box: the i8 MFMA layout probe, the GPU suite (or a subset: PYTEST_K), then
# round-only bench runs alternating the arms (ARMS="A B C", ARM_<x> = env assignments, default: the
# VALU base conversions vs the matrix-core ones).  Stops at the first crash or time limit.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-ab}
ARM_A=${ARM_A:-AESFHE_BCONV_VALU=1}
ARM_B=${ARM_B:-AESFHE_BCONV_VALU=0}
REPS=${REPS:-2}
BENCH_ARGS=${BENCH_ARGS:---steps 5 --warmup 1 --no-configs --no-harness --client-batch 0 --aes10-batch 0 --no-cpu-baseline --config5 off}
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
if [ -x tools/mfma_i8_probe ] && [ -z "$NO_PROBE" ]; then
  timeout -k 10 60 ./tools/mfma_i8_probe > gpurun_out/${TAG}_probe.log 2>&1; rc=$?; cat gpurun_out/${TAG}_probe.log; fatal $rc probe
fi
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu ${PYTEST_K:+-k "$PYTEST_K"} --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
  tail -15 gpurun_out/${TAG}_pytest.log; fatal $rc pytest
fi
if [ -n "$EXTRA_TEST_ENV" ]; then  # the parity subset again under another switch (e.g. AESFHE_KS_PIPE=1)
  env $EXTRA_TEST_ENV timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_aes128_full.py tests/test_bootstrap.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_extra.log 2>&1; rc=$?
  tail -5 gpurun_out/${TAG}_pytest_extra.log; fatal $rc pytest_extra
fi
ARMS=${ARMS:-A B}
for i in $(seq 1 $REPS); do
  for arm in $ARMS; do
    eval "ARMV=\$ARM_$arm"
    env $ARMV timeout -k 10 600 python -u bench.py $BENCH_ARGS > gpurun_out/${TAG}_${arm}${i}.json 2> gpurun_out/${TAG}_${arm}${i}.err; rc=$?
    fatal $rc "bench $arm$i"
    [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_${arm}${i}.err; continue; }
    python3 tools/brief.py gpurun_out/${TAG}_${arm}${i}.json "$arm$i" modup moddown ks_rows_fin ntt_fwd_cols
  done
done
