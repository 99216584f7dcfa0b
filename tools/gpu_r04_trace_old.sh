#!/bin/bash
# tools/aes10_trace.py with $OLDLIB for SEEDS (margins per step, for comparison), own time limit per run.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-tro}
export AESFHE_LIB=$GRAFT_REPO_ROOT/$OLDLIB
for s in ${SEEDS:-1}; do
  timeout -k 10 300 python3 -u tools/aes10_trace.py $s > gpurun_out/${TAG}_$s.log 2>&1 || { tail -20 gpurun_out/${TAG}_$s.log; exit 1; }
  echo "seed $s $OLDLIB"; grep -v amdgpu.ids gpurun_out/${TAG}_$s.log | tail -8
done
