set -o pipefail
mkdir -p gpurun_out/kab
timeout -k 10 300 python bench.py --no-cpu-baseline --aes10-batch 0 --special-primes 10 --check > gpurun_out/kab/k10c.json 2> gpurun_out/kab/k10c.err || exit 1
for i in 1 2; do for K in 8 10; do
timeout -k 10 300 python bench.py --no-cpu-baseline --aes10-batch 0 --special-primes $K > gpurun_out/kab/k$K.$i.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/kab/k$K.$i.json')); print('K$K', d['value'])"
done; done
timeout -k 10 400 python bench.py --no-cpu-baseline --special-primes 10 --check > gpurun_out/kab/k10_aes10.json 2> gpurun_out/kab/k10_aes10.err || exit 1
