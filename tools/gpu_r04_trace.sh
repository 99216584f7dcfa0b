#!/bin/bash
# tools/aes10_trace.py for SEEDS with the current library; a seed that ends wrong is re-run with
# $OLDLIB.  Each run under its own time limit.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-tr}
for s in ${SEEDS:-1 2 3}; do
  unset AESFHE_LIB
  timeout -k 10 300 python3 -u tools/aes10_trace.py $s > gpurun_out/${TAG}_new_$s.log 2>&1 || { tail -20 gpurun_out/${TAG}_new_$s.log; exit 1; }
  echo "seed $s new"; grep -v "wrong blocks    0" gpurun_out/${TAG}_new_$s.log | grep -v amdgpu.ids
  if grep -q "ok False" gpurun_out/${TAG}_new_$s.log && [ -n "$OLDLIB" ]; then
    export AESFHE_LIB=$GRAFT_REPO_ROOT/$OLDLIB
    timeout -k 10 300 python3 -u tools/aes10_trace.py $s > gpurun_out/${TAG}_old_$s.log 2>&1 || { tail -20 gpurun_out/${TAG}_old_$s.log; exit 1; }
    echo "seed $s old"; grep -v "wrong blocks    0" gpurun_out/${TAG}_old_$s.log | grep -v amdgpu.ids
  fi
done
