#!/bin/bash
# Cleaning before the last refresh: per-step margins (tools/aes10_trace.py, SEEDS), the GPU tests of
# the ten-round paths, then the bench's ten-round leg RUNS times; own time limit per step.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-cl}
for s in ${SEEDS:-1 2}; do
  timeout -k 10 300 python3 -u tools/aes10_trace.py $s > gpurun_out/${TAG}_trace_$s.log 2>&1 || { tail -20 gpurun_out/${TAG}_trace_$s.log; exit 1; }
  echo "seed $s"; grep -v amdgpu.ids gpurun_out/${TAG}_trace_$s.log | tail -9
done
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -k "${K:-aes128 or config4 or bootstrap}" --timeout 400 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
B="python3 bench.py --steps 1 --warmup 0 --no-configs --no-harness --client-batch 0 --no-cpu-baseline --config5 off --profile-steps 0"
for n in $(seq 1 ${RUNS:-3}); do
  timeout -k 10 300 $B > gpurun_out/${TAG}_a10_${n}.json 2> gpurun_out/${TAG}_a10_${n}.err || { tail -20 gpurun_out/${TAG}_a10_${n}.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); a=d['aes128_10_rounds']; print(a['value'], a['verified'], a.get('mismatch'), a['bootstrap_cts_groups'])" gpurun_out/${TAG}_a10_${n}.json
done
