#!/bin/bash
# The bench's ten-round leg alone (its default 16 sets, FIPS-checked with mismatch details), run
# N times in separate processes, alternating the current library with $OLDLIB when given; each
# run under its own time limit.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-a10}
B="python3 bench.py --steps 1 --warmup 0 --no-configs --no-harness --client-batch 0 --no-cpu-baseline --config5 off --profile-steps 0"
for n in $(seq 1 ${RUNS:-2}); do
  for lib in new ${OLDLIB:+old}; do
    if [ $lib = old ]; then export AESFHE_LIB=$GRAFT_REPO_ROOT/$OLDLIB; else unset AESFHE_LIB; fi
    timeout -k 10 400 $B > gpurun_out/${TAG}_${lib}_${n}.json 2> gpurun_out/${TAG}_${lib}_${n}.err || { tail -20 gpurun_out/${TAG}_${lib}_${n}.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); a=d['aes128_10_rounds']; print(sys.argv[2], a['value'], a['verified'], a.get('mismatch'))" gpurun_out/${TAG}_${lib}_${n}.json $lib
  done
done
