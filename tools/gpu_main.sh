#!/bin/bash
# GPU session: GPU tests, smoke, the default bench, config 5's shard (round + 10-round), and a
# rocprofv3 kernel summary of the default round (--aes10-batch 0).  Each GPU step has its own
# limit; steps are chained with && (a failure or time-out ends the script).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-main}
C5="--log-n 17 --max-level 35 --special-primes 12 --scale-bits 44 --batch 16 --aes10-batch 16 --no-cpu-baseline --no-configs"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1 \
 && echo "gpu tests ok" \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 \
 && echo "smoke ok" \
 && timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
 && echo "bench ok" \
 && if [ -z "$NO_C5" ]; then timeout -k 10 900 python bench.py $C5 --steps 2 --warmup 1 > gpurun_out/bench_c5_${TAG}.json 2> gpurun_out/bench_c5_${TAG}.err && echo "config5 ok"; fi \
 && if [ -n "$PROF" ]; then timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o bench -- python bench.py --no-cpu-baseline --no-configs --aes10-batch 0 ${BENCH_ARGS} > gpurun_out/prof_${TAG}.log 2>&1 && rm -f gpurun_out/prof_${TAG}/*_kernel_trace.csv && echo "rocprof ok"; fi
rc=$?
tail -3 gpurun_out/pytest_gpu_${TAG}.log; tail -1 gpurun_out/smoke_${TAG}.log
python3 - "$TAG" <<'PY'
import json, sys
t = sys.argv[1]
for f in (f"gpurun_out/bench_{t}.json", f"gpurun_out/bench_c5_{t}.json"):
    try:
        r = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as ex:
        print(f, "missing", ex); continue
    a = r.get("aes128_10_rounds") or {}
    print(f, r["value"], r["config"]["verified"], r["roofline"]["frac"], "aes10", a.get("value"), a.get("verified"), a.get("timed_mallocs"))
PY
exit $rc
