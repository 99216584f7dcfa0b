#!/bin/bash
# tools/aes10_trace.py with the pool poisoned (AESFHE_POOL_POISON=1), current library then $OLDLIB
# (built before the poison switch existed: unpoisoned, for reference); own time limit per run.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-po}
for s in ${SEEDS:-1}; do
  AESFHE_POOL_POISON=1 timeout -k 10 300 python3 -u tools/aes10_trace.py $s ${SETS:-16} > gpurun_out/${TAG}_new_$s.log 2>&1 || { tail -20 gpurun_out/${TAG}_new_$s.log; exit 1; }
  echo "seed $s new (poisoned)"; grep -v amdgpu.ids gpurun_out/${TAG}_new_$s.log | head -30
done
