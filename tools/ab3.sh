#!/bin/bash
# A/B/C... of engine builds (AESFHE_LIB) on the headline round, alternated to cancel drift:
#   tools/ab3.sh "<libA> <libB> ..." [bench args]
set -o pipefail
mkdir -p gpurun_out/ab
LIBS=$1; shift
for i in 1 2; do
  for lib in $LIBS; do
    v=$(basename $lib .so)
    AESFHE_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --aes10-batch 0 "$@" > gpurun_out/ab/$v.$i.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab/$v.$i.json')); print('$v', $i, d['value'], d['roofline']['keyswitch_kernels_gbs'])"
  done
done
