#!/bin/bash
# rocprofv3 --kernel-trace --stats of the bench's round alone (the line's roofline kernel average
# must agree with the summary's), then the same for the ten-round leg; each step time-limited.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-rp}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_round_${TAG} -o round -- python3 bench.py --steps 5 --warmup 1 --aes10-batch 0 --no-configs --no-harness --client-batch 0 --no-cpu-baseline --config5 off > gpurun_out/prof_round_${TAG}.json 2> gpurun_out/prof_round_${TAG}.err \
 && rm -f gpurun_out/prof_round_${TAG}/*_kernel_trace.csv && echo "round profiled" \
 && timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof10_${TAG} -o aes10 -- python3 bench.py --steps 1 --warmup 1 --no-configs --no-harness --client-batch 0 --no-cpu-baseline --config5 off > gpurun_out/prof10_${TAG}.json 2> gpurun_out/prof10_${TAG}.err \
 && rm -f gpurun_out/prof10_${TAG}/*_kernel_trace.csv && echo "aes10 profiled"
