#!/bin/bash
# A/B of the bit-mode bootstrap: bits_opt (default) vs --no-opt, timings + phases, then a
# rocprofv3 kernel summary of each (GPU box)
set -o pipefail
mkdir -p gpurun_out/bootab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$PYTEST_FILES" ]; then
  timeout -k 10 600 python -u -m pytest $PYTEST_FILES -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/bootab/pytest.log 2>&1 || { tail -30 gpurun_out/bootab/pytest.log; exit 1; }
  tail -3 gpurun_out/bootab/pytest.log
fi
for v in opt noopt opt2; do
  f=""; [ $v = noopt ] && f="--no-opt"
  timeout -k 10 300 python -u tools/boot_bench.py --scale-bits 40 --special-primes 10 --batch ${PPC:-16} --phases $f > gpurun_out/bootab/$v.log 2>&1 || { tail -20 gpurun_out/bootab/$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/bootab/$v.log
done
for v in opt noopt; do
  f=""; [ $v = noopt ] && f="--no-opt"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bootab/prof_$v -o b -- python3 tools/boot_bench.py --scale-bits 40 --special-primes 10 --batch ${PPC:-16} --reps 2 $f > gpurun_out/bootab/prof_$v.log 2>&1 || { tail -20 gpurun_out/bootab/prof_$v.log; exit 1; }
done
echo done
