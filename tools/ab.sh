#!/bin/bash
# A/B of two engine builds (AESFHE_LIB) on the headline round, alternated to cancel drift:
#   tools/ab.sh <libA> <libB> [bench args]
set -o pipefail
mkdir -p gpurun_out/ab
A=$1; B=$2; shift 2
for i in 1 2; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    AESFHE_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --aes10-batch 0 "$@" > gpurun_out/ab/$v$i.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab/$v$i.json')); print('$v$i', d['value'])"
  done
done
