#!/bin/bash
# SlotToCoeff BSGS split: the bit bootstrap at the bench's parameters (64 bit ciphertexts per
# call, 5-map CtS) with stc_baby_scale 2 (default) / 1 / 0.5 / 2, phases per run.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
n=0
for sc in ${SCALES:-2 4 8 2 4}; do
  n=$((n+1))
  timeout -k 10 300 python3 -u tools/boot_bench.py --scale-bits 40 --special-primes 10 --digit-primes 12 --batch 32 --reps 3 --phases --cts-groups 5 --stc-baby-scale $sc > gpurun_out/stcab_${n}_$sc.log 2>&1 || { tail -5 gpurun_out/stcab_${n}_$sc.log; exit 1; }
  python3 -c "
import json; L=[json.loads(l) for l in open('gpurun_out/stcab_${n}_$sc.log') if l.startswith('{')]
p=L[1]['phases_ms']; print('stc_baby_scale $sc', L[0]['ms_per_call'], L[0]['max_err'], 'stc', round(p['stc0']+p['stc1']+p['stc2'],2), p['stc0'], p['stc1'], p['stc2'])"
done
