#!/bin/bash
# Bit-mode bootstrap per CoeffToSlot group count (N = 2^16, L = 30, K = 10, alpha = 12, scale 40,
# 32 pairs per call as in the ten-round leg): time per call and per phase.  Each step limited.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-cg}
A="--scale-bits 40 --special-primes 10 --digit-primes 12 --batch ${BATCH:-32} --reps 2 --phases"
for g in ${GROUPS_LIST:-3 4 5}; do
  timeout -k 10 300 python tools/boot_bench.py $A --cts-groups $g > gpurun_out/boot_${TAG}_g$g.json 2> gpurun_out/boot_${TAG}_g$g.err || { echo "groups $g failed"; tail -5 gpurun_out/boot_${TAG}_g$g.err; exit 1; }
  echo "groups $g:"; cat gpurun_out/boot_${TAG}_g$g.json
done
