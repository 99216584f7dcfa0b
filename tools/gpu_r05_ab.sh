#!/bin/bash
# Round 5 A/B on one box: the i8 MFMA layout probe, the GPU suite (or a subset: PYTEST_K), then
# round-only bench runs alternating the two arms (ARM_A / ARM_B env assignments, default: the
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
for i in $(seq 1 $REPS); do
  for arm in A B; do
    eval "ARMV=\$ARM_$arm"
    env $ARMV timeout -k 10 600 python -u bench.py $BENCH_ARGS > gpurun_out/${TAG}_${arm}${i}.json 2> gpurun_out/${TAG}_${arm}${i}.err; rc=$?
    fatal $rc "bench $arm$i"
    [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_${arm}${i}.err; continue; }
    python3 tools/brief.py gpurun_out/${TAG}_${arm}${i}.json "$arm$i" modup moddown ks_rows_fin ntt_fwd_cols
  done
done
