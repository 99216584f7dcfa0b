#!/bin/bash
# A/B of an environment setting on the headline round, alternated: tools/ab_env.sh "VAR=a VAR=b" [bench args]
set -o pipefail
mkdir -p gpurun_out/ab_env
SETS=$1; shift
for i in 1 2; do
  for s in $SETS; do
    env $s timeout -k 10 300 python bench.py --no-cpu-baseline --aes10-batch 0 "$@" > gpurun_out/ab_env/$s.$i.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_env/$s.$i.json')); print('$s', $i, d['value'], d['roofline']['frac'], d['config'].get('verified'))"
  done
done
