#!/bin/bash
# Kernel-level profile of the bench round (dev loop): rocprofv3 stats of tools/round_stages.py.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
B=${B:-16}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rows -o rows -- python3 tools/round_stages.py rows $B > gpurun_out/prof_rows.log 2>&1
rc=$?; grep -v "^W2\|^E2" gpurun_out/prof_rows.log | tail -6; exit $rc
