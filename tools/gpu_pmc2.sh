#!/bin/bash
# PMC passes over tools/ks_driver (N = 2^16, L = 30 multiplies: every NTT and key-switch kernel),
# one counter per run, --kernel-trace only (no sys/runtime traces): FETCH_SIZE and WRITE_SIZE
# for the NTT traffic ratio (tools/ntt_traffic.py), then SQ wait counters.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-p2}
run() { local n=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_$n -o p -- ./tools/ks_driver 16 4 > gpurun_out/pmc_${TAG}_$n.log 2>&1; }
run fetch FETCH_SIZE && run write WRITE_SIZE && run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU
rc=$?
find gpurun_out/pmc_${TAG}_* -name "*counter_collection*.csv" | head
exit $rc
