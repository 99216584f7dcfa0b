#!/bin/bash
# GPU session: batch-size sweep of the round (--batch) and of the bootstrap batch (--aes10-ppc).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-sw}
Q="--no-configs --no-cpu-baseline --profile-steps 0"
for b in ${BATCHES:-40 48}; do
  timeout -k 10 600 python bench.py $Q --aes10-batch 0 --batch $b > gpurun_out/sweep_${TAG}_b$b.json 2> gpurun_out/sweep_${TAG}_b$b.err || exit $?
  echo "batch $b: $(cut -c1-160 gpurun_out/sweep_${TAG}_b$b.json)"
done
for p in ${PPCS:-4}; do
  timeout -k 10 600 python bench.py $Q --batch 8 --steps 1 --aes10-ppc $p > gpurun_out/sweep_${TAG}_p$p.json 2> gpurun_out/sweep_${TAG}_p$p.err || exit $?
  python3 -c "import json;r=json.loads(open('gpurun_out/sweep_${TAG}_p$p.json').read());a=r['aes128_10_rounds'];print('ppc $p', a['value'], a['verified'], a['bootstrap_ms_per_bit_ct'], a['timed_mallocs'], a['pool']['held'])"
done
