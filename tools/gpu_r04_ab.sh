#!/bin/bash
# Generic A/B of an engine env switch on the bench round: parity tests selected by -k "$K", then
# the round with $VAR=1 / 0 alternated (the first run of a fresh box is discarded: warm-up).
# VAR=AESFHE_X K="expr" TAG=t bash tools/gpu_r04_ab.sh
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-ab}
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest tests/ -x -q -m gpu -k "$K" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest.log
fi
B="python3 bench.py --steps 3 --warmup 1 --no-configs --no-harness --client-batch 0 --aes10-batch ${AES10:-0} --no-cpu-baseline --config5 off"
n=0
for arm in 0 1 0 1 0; do
  n=$((n+1))
  env $VAR=$arm timeout -k 10 400 $B > gpurun_out/${TAG}_${n}_v$arm.json 2> gpurun_out/${TAG}_${n}_v$arm.err || { tail -20 gpurun_out/${TAG}_${n}_v$arm.err; exit 1; }
  python3 tools/brief.py gpurun_out/${TAG}_${n}_v$arm.json "$VAR=$arm" ${PATS:-ntt_fwd_cols modup}
done
