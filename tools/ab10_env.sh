#!/bin/bash
# A/B of environment settings on the 10-round AES-128 workload, alternated:
#   tools/ab10_env.sh "VAR=a VAR=b" [bench args]
set -o pipefail
mkdir -p gpurun_out/ab10_env
SETS=$1; shift
for i in 1 2; do
  for s in $SETS; do
    env $s timeout -k 10 400 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --check "$@" > gpurun_out/ab10_env/$s.$i.json 2>gpurun_out/ab10_env/$s.$i.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab10_env/$s.$i.json')); a=d['aes128_10_rounds']; print('$s', $i, d['value'], a['value'], a['verified'])"
  done
done
