#!/bin/bash
# A/B of the LDS-resident ModUp + column-pass fusion (tools/modup_cols_bench.hip, built in-tree):
# timings at B = 16 / 32, a kernel summary and FETCH_SIZE / WRITE_SIZE passes (GPU box)
set -o pipefail
mkdir -p gpurun_out/modupab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for b in 16 32; do
  timeout -k 10 120 ./tools/modup_cols_bench $b 10 | tee -a gpurun_out/modupab/times.json || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/modupab/trace -o t -- ./tools/modup_cols_bench 32 3 > gpurun_out/modupab/trace.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/modupab/fetch -o f -- ./tools/modup_cols_bench 32 1 > gpurun_out/modupab/fetch.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/modupab/write -o w -- ./tools/modup_cols_bench 32 1 > gpurun_out/modupab/write.log 2>&1 || exit 1
echo done
