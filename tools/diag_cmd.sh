set -o pipefail
mkdir -p gpurun_out
for a in "16 30 8 40 50" "16 30 8 44 50" "16 30 8 40 45" "16 30 8 40 47"; do
  timeout -k 10 300 python tools/boot_general_diag.py $a >> gpurun_out/bootgen.log 2>&1 || exit 1
done
grep -v amdgpu gpurun_out/bootgen.log
