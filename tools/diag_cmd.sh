set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_services.py -v -s --timeout 500 --timeout-method thread -k "gf_mul2 or mixrow or transformer" > gpurun_out/svc_gpu.log 2>&1
grep -E "PASS|FAIL|MixRow" gpurun_out/svc_gpu.log
for a in "16 30 8 40 50" "16 30 8 44 50" "16 30 8 40 45"; do
  timeout -k 10 300 python tools/boot_general_diag.py $a >> gpurun_out/bootgen.log 2>&1 || exit 1
done
grep -v amdgpu gpurun_out/bootgen.log
timeout -k 10 900 python bench.py --log-n 17 --max-level 35 --special-primes 12 --scale-bits 44 --batch 16 --aes10-batch 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err; rc=$?
tail -4 gpurun_out/bench_c5.err; cat gpurun_out/bench_c5.json
exit $rc
