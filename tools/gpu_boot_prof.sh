#!/bin/bash
# bootstrap timing at a few batch sizes + a rocprofv3 kernel profile of the batch-8 call (GPU box)
set -o pipefail
mkdir -p gpurun_out/bootprof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/boot_times.log
: > $out
for b in 8; do
  timeout -k 10 300 python tools/boot_bench.py --scale-bits ${SB:-40} --batch $b --phases >> $out 2>&1 || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bootprof -o boot -- python3 tools/boot_bench.py --scale-bits ${SB:-40} --batch 8 --reps 1 > gpurun_out/bootprof.log 2>&1 || exit 1
