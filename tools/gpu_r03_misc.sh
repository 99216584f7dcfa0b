#!/bin/bash
# (1) bench.py under torchrun with 2 ranks sharing the box's one GPU (gloo: shared seed, key
# fingerprint, scatter/gather with host staging), small batch; (2) the ten-round leg at 4 pairs
# per bootstrap call.  Steps chained with &&, each limited.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --batch 4 --aes10-batch 0 --no-cpu-baseline --no-configs --no-harness --client-batch 0 > gpurun_out/rehearsal2.json 2> gpurun_out/rehearsal2.err \
 && echo "rehearsal ok" && tail -c 600 gpurun_out/rehearsal2.json \
 && timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --no-configs --no-harness --client-batch 0 --no-cpu-baseline --aes10-ppc 4 > gpurun_out/ppc4.json 2> gpurun_out/ppc4.err \
 && echo "ppc4 ok"
rc=$?
tail -3 gpurun_out/rehearsal2.err; tail -3 gpurun_out/ppc4.err 2>/dev/null
exit $rc
