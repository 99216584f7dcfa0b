#!/bin/bash
# Kernel mix of the bit-mode bootstrap at the bench's parameters (N = 2^16, L = 30, K = 10,
# alpha = 12, 64 bit ciphertexts per call, 5-map CtS): rocprofv3 summary of tools/boot_bench.py
# (setup + 1 warm-up + 2 timed calls), then the phase split without the profiler.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-bootprof}
G=${CTSG:-5}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o boot -- python3 tools/boot_bench.py --scale-bits 40 --special-primes 10 --digit-primes 12 --batch 32 --reps 2 --cts-groups $G > gpurun_out/${TAG}_prof.log 2>&1 \
 && rm -f gpurun_out/${TAG}_prof/*_kernel_trace.csv && echo "profiled" \
 && timeout -k 10 300 python3 -u tools/boot_bench.py --scale-bits 40 --special-primes 10 --digit-primes 12 --batch 32 --reps 2 --phases --cts-groups $G > gpurun_out/${TAG}_phases.log 2>&1 \
 && cat gpurun_out/${TAG}_phases.log
