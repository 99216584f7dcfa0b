#!/bin/bash
# bootstrap precision / speed vs scale bits and batch, plus the round time per scale (GPU box)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/boot_sweep.log
: > $out
for sb in 41 42 44; do
  for b in 1 8; do
    timeout -k 10 300 python tools/boot_bench.py --scale-bits $sb --batch $b >> $out 2>&1 || exit 1
  done
  SCALE_BITS=$sb timeout -k 10 300 python tools/round_stages.py rows 16 >> $out 2>&1 || exit 1
done
