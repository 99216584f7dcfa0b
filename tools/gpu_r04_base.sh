#!/bin/bash
# Round-4 baseline measurements of HEAD: (1) rocprofv3 kernel summary of the ten-round leg
# (the bench's round step + aes128_10_rounds), (2) one refresh's phase split at 64 ciphertexts
# per call for the 5-map and the 3-map CoeffToSlot bootstrappers.  Steps chained, each limited.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-base}
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof10_${TAG} -o aes10 -- python3 bench.py --steps 1 --warmup 1 --no-configs --no-harness --client-batch 0 --no-cpu-baseline > gpurun_out/prof10_${TAG}.json 2> gpurun_out/prof10_${TAG}.err \
 && rm -f gpurun_out/prof10_${TAG}/*_kernel_trace.csv && echo "aes10 profiled" \
 && timeout -k 10 300 python3 -u tools/boot_bench.py --scale-bits 40 --special-primes 10 --digit-primes 12 --batch 32 --reps 2 --phases --cts-groups 5 > gpurun_out/boot5_${TAG}.log 2>&1 \
 && timeout -k 10 300 python3 -u tools/boot_bench.py --scale-bits 40 --special-primes 10 --digit-primes 12 --batch 32 --reps 2 --phases --cts-groups 3 > gpurun_out/boot3_${TAG}.log 2>&1 \
 && echo "phases ok"
rc=$?
tail -3 gpurun_out/prof10_${TAG}.err; cat gpurun_out/boot5_${TAG}.log gpurun_out/boot3_${TAG}.log 2>/dev/null
exit $rc
