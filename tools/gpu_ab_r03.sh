#!/bin/bash
# A/B of two product builds on one box: OLD=aes-fhe_amd/build/ab_old.so vs the in-tree library,
# alternated (A B A B), the round bench only; optional GPU tests first (PYTEST_FILES / PYTEST_K).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-ab}
ARGS="--steps 4 --warmup 1 --no-configs --aes10-batch 0 --no-cpu-baseline --client-batch 0 --no-harness ${AB_ARGS}"
if [ -n "$PYTEST_FILES" ]; then
  timeout -k 10 600 python -u -m pytest $PYTEST_FILES -x -v -m gpu --timeout 400 --timeout-method thread ${PYTEST_K} > gpurun_out/pytest_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
  echo "gpu tests ok"; tail -1 gpurun_out/pytest_${TAG}.log
fi
for r in 1 2; do
  AESFHE_LIB=aes-fhe_amd/build/ab_old.so timeout -k 10 300 python bench.py $ARGS > gpurun_out/${TAG}_A$r.json 2> gpurun_out/${TAG}_A$r.err || exit 1
  timeout -k 10 300 python bench.py $ARGS > gpurun_out/${TAG}_B$r.json 2> gpurun_out/${TAG}_B$r.err || exit 1
  echo "round $r done"
done
python3 - "$TAG" <<'PY'
import json, sys
t = sys.argv[1]
for v in ("A1", "B1", "A2", "B2"):
    r = json.loads(open(f"gpurun_out/{t}_{v}.json").read().strip().splitlines()[-1])
    k = r["roofline"]["kernels"]
    top = {n: k[n]["avg_us"] for n in list(k)[:8]}
    print(v, r["value"], r["ms_per_step"], r["config"]["verified"], top)
PY
