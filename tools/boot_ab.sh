#!/bin/bash
# A/B of engine builds on bit-mode bootstrapping (tools/boot_bench.py), alternated:
#   tools/boot_ab.sh "<libA> <libB> ..." [boot_bench args]
set -o pipefail
mkdir -p gpurun_out/boot_ab
LIBS=$1; shift
for i in 1 2; do
  for lib in $LIBS; do
    v=$(basename $lib .so)
    AESFHE_LIB=$lib timeout -k 10 300 python tools/boot_bench.py "$@" > gpurun_out/boot_ab/$v.$i.json 2>/dev/null || exit 1
    echo "$v $i $(head -c 400 gpurun_out/boot_ab/$v.$i.json)"
  done
done
