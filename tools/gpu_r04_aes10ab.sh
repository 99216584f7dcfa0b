#!/bin/bash
# The bench's ten-round leg alone (default 16 sets, mismatch details), RUNS times per arm of the
# env switch $VAR (1, 0 alternated), each run in its own process under its own time limit.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-a10ab}
B="python3 bench.py --steps 1 --warmup 0 --no-configs --no-harness --client-batch 0 --no-cpu-baseline --config5 off --profile-steps 0"
for n in $(seq 1 ${RUNS:-4}); do
  for arm in 1 0; do
    env $VAR=$arm timeout -k 10 300 $B > gpurun_out/${TAG}_${arm}_${n}.json 2> gpurun_out/${TAG}_${arm}_${n}.err || { tail -20 gpurun_out/${TAG}_${arm}_${n}.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); a=d['aes128_10_rounds']; print(sys.argv[2], d['value'], d['config']['verified'], a['value'], a['verified'], a.get('mismatch'))" gpurun_out/${TAG}_${arm}_${n}.json "$VAR=$arm"
  done
done
