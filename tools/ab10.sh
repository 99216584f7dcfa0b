#!/bin/bash
# A/B of two engine builds (AESFHE_LIB) on the 10-round AES-128 workload (with bootstrapping),
# alternated; GPU tests on the current build first:  tools/ab10.sh <libA> <libB> [bench args]
set -o pipefail
mkdir -p gpurun_out/ab10
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A=$1; B=$2; shift 2
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab10/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/ab10/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/ab10/pytest_gpu.log
for i in 1 2; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    AESFHE_LIB=$lib timeout -k 10 400 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --check "$@" > gpurun_out/ab10/$v$i.json 2>gpurun_out/ab10/$v$i.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab10/$v$i.json')); a=d['aes128_10_rounds']; print('$v$i', d['value'], a['value'], a['verified'], a['bootstrap_share'])"
  done
done
