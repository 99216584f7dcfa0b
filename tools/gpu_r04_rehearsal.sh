#!/bin/bash
# bench.py --gpus 2 WITHOUT torchrun on the 1-GPU box: the launcher starts two ranks (children of
# torch.distributed.run); they share the GPU, so the backend is gloo (RCCL needs a GPU per rank);
# small batch so both engines fit.  The line must say n_gpus 2 and scatter_gather verified.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 bench.py --gpus 2 --steps 2 --warmup 1 --batch 4 --aes10-batch 0 --no-configs --no-harness --client-batch 0 --no-cpu-baseline --launch-timeout 500 > gpurun_out/rehearsal2.json 2> gpurun_out/rehearsal2.err
rc=$?
tail -4 gpurun_out/rehearsal2.err
[ $rc -eq 0 ] && python3 -c "
import json; d=json.loads(open('gpurun_out/rehearsal2.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'devices', d['visible_devices'], 'value', d['value'], 'verified', d['config']['verified'])
print(d['scatter_gather'])"
exit $rc
