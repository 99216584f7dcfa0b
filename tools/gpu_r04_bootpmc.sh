#!/bin/bash
# HBM bytes and durations per kernel class of the bit bootstrap (tools/boot_bench.py at the bench's
# parameters, 64 bit ciphertexts per call, 5-map CtS): FETCH_SIZE and WRITE_SIZE passes with the
# kernel trace kept (durations per dispatch), summarised by tools/boot_pmc.py.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BB="tools/boot_bench.py --scale-bits 40 --special-primes 10 --digit-primes 12 --batch 32 --reps 2 --cts-groups 5"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/bpmc_fetch -o p -- python3 $BB > gpurun_out/bpmc_fetch.log 2>&1 \
 && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/bpmc_write -o p -- python3 $BB > gpurun_out/bpmc_write.log 2>&1 \
 && python3 tools/boot_pmc.py gpurun_out/bpmc_fetch gpurun_out/bpmc_write
