#!/bin/bash
# Round-end evidence on the current tree: the GPU suite, smoke, the driver's bench command, then
# rocprofv3 --kernel-trace --stats of the bench's round alone (profiles/r06/round_kernel_stats.csv).
# The PMC passes are tools/gpu_r06_pmc.sh (separate call).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-fin}
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
  python3 tools/brief.py gpurun_out/${T}_bench.json bench ks_rows_fin ntt_fwd_cols poly2 modup moddown
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o round -- python3 bench.py --steps 5 --warmup 1 --aes10-batch 0 --no-configs --no-harness --client-batch 0 --no-cpu-baseline --config5 off > gpurun_out/${T}_prof.json 2> gpurun_out/${T}_prof.err \
 && rm -f gpurun_out/${T}_prof/*_kernel_trace.csv && echo "round profiled" \
 && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_aprof -o aes10 -- python3 bench.py --steps 1 --warmup 0 --profile-steps 0 --no-configs --no-harness --client-batch 0 --no-cpu-baseline --config5 off > gpurun_out/${T}_aprof.json 2> gpurun_out/${T}_aprof.err \
 && rm -f gpurun_out/${T}_aprof/*_kernel_trace.csv && echo "ten rounds profiled"
