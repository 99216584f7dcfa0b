#!/bin/bash
# Final round-3 measurement of the benched tree: a rocprofv3 kernel summary of the bench's round
# (the command whose NTT launches the bench line's roofline averages), then the PMC passes over
# one round step (tools/gpu_r03_pmc.sh, no bench).  Steps chained with &&, each limited.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-fin}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o round -- python3 bench.py --steps 3 --warmup 1 --no-configs --no-harness --client-batch 0 --aes10-batch 0 --no-cpu-baseline > gpurun_out/prof_${TAG}.json 2> gpurun_out/prof_${TAG}.err \
 && rm -f gpurun_out/prof_${TAG}/*_kernel_trace.csv && echo "round profiled" \
 && NO_BENCH=1 TAG=${TAG} bash tools/gpu_r03_pmc.sh
