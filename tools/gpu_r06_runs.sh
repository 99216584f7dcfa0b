#!/bin/bash
# Round 6: probe, a pytest selection, then a list of bench runs, one per line of $RUNS:
#   name|ENV=v ENV2=v|bench args
# (round-only / ten-round-only arms for A/B).  Stops at the first crash or time limit.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r6}
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
if [ -x tools/mfma_i8_probe ] && [ -z "$NO_PROBE" ]; then
  timeout -k 10 60 ./tools/mfma_i8_probe > gpurun_out/${TAG}_probe.log 2>&1; rc=$?; cat gpurun_out/${TAG}_probe.log; fatal $rc probe
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
  tail -6 gpurun_out/${TAG}_pytest.log; fatal $rc pytest
  [ $rc -ne 0 ] && [ -n "$STOP_ON_FAIL" ] && exit 1
fi
if [ -n "$EXTRA_TESTS" ]; then  # the same selection again under an opt-in env (EXTRA_TEST_ENV)
  env $EXTRA_TEST_ENV timeout -k 10 900 python -u -m pytest $EXTRA_TESTS -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_extra.log 2>&1; rc=$?
  tail -6 gpurun_out/${TAG}_pytest_extra.log; fatal $rc pytest_extra
  [ $rc -ne 0 ] && [ -n "$STOP_ON_FAIL" ] && exit 1
fi
ROUND="--steps 5 --warmup 1 --no-configs --no-harness --client-batch 0 --aes10-batch 0 --no-cpu-baseline --config5 off"
AES10="--steps 1 --warmup 0 --profile-steps 0 --no-configs --no-harness --client-batch 0 --no-cpu-baseline --config5 off"
while IFS='|' read -r name envs args; do
  [ -z "$name" ] && continue
  args=${args//@ROUND/$ROUND}
  args=${args//@AES10/$AES10}
  env $envs timeout -k 10 600 python -u bench.py $args > gpurun_out/${TAG}_${name}.json 2> gpurun_out/${TAG}_${name}.err; rc=$?
  fatal $rc "bench $name"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_${name}.err; continue; }
  python3 tools/brief.py gpurun_out/${TAG}_${name}.json "$name" ${BRIEF:-modup moddown ks_rows_fin ntt_fwd_cols bsgs dot_pt ks_inner}
done <<< "$RUNS"
