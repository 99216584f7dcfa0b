#!/bin/bash
# The bench's ten-round leg at pairs-per-call PPCS (alternated, RUNS each), own time limit per run.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-ppc}
B="python3 bench.py --steps 1 --warmup 0 --no-configs --no-harness --client-batch 0 --no-cpu-baseline --config5 off --profile-steps 0"
for n in $(seq 1 ${RUNS:-2}); do
  for p in ${PPCS:-4 8}; do
    timeout -k 10 300 $B --aes10-ppc $p > gpurun_out/${TAG}_${p}_${n}.json 2> gpurun_out/${TAG}_${p}_${n}.err || { tail -20 gpurun_out/${TAG}_${p}_${n}.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); a=d['aes128_10_rounds']; print('ppc', sys.argv[2], a['value'], a['verified'], a['bootstrap_share'], round(a['pool']['peak_live']/1e9,1))" gpurun_out/${TAG}_${p}_${n}.json $p
  done
done
