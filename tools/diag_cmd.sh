set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/aes10_diag.py 17 35 12 44 > gpurun_out/aes10diag17.log 2>&1; rc=$?
timeout -k 10 400 python tools/aes10_diag.py 17 35 12 40 > gpurun_out/aes10diag17s40.log 2>&1
cat gpurun_out/aes10diag17.log gpurun_out/aes10diag17s40.log | tail -40
exit $rc
