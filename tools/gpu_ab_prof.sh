#!/bin/bash
# One GPU session for a kernel change: GPU tests on the current build, an alternated A/B of the
# headline round (old vs new library), and rocprofv3 kernel stats of one round with each library.
#   tools/gpu_ab_prof.sh <libOld> <libNew> [bench args]
set -o pipefail
mkdir -p gpurun_out/abp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A=$1; B=$2; shift 2
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/abp/pytest_gpu.log 2>&1 \
 && echo "gpu tests ok" && tail -1 gpurun_out/abp/pytest_gpu.log \
 && bash tools/ab.sh "$A" "$B" "$@" \
 && for v in A B; do
      lib=$A; [ $v = B ] && lib=$B
      AESFHE_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abp/prof_$v -o k -- python bench.py --no-cpu-baseline --aes10-batch 0 --steps 1 --warmup 1 "$@" > gpurun_out/abp/prof_$v.log 2>&1 || exit 1
    done \
 && python tools/cmpk.py gpurun_out/abp/prof_A/k_kernel_stats.csv gpurun_out/abp/prof_B/k_kernel_stats.csv
rc=$?
tail -3 gpurun_out/abp/pytest_gpu.log
exit $rc
