set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "linear_bsgs or full_params" --timeout 300 --timeout-method thread > gpurun_out/pt_lin.log 2>&1; rc=$?; tail -n 3 gpurun_out/pt_lin.log; [ $rc = 0 ] || exit 1
bash tools/boot_ab.sh "${LIBS:-aes-fhe_amd/build/libaesfhe_o.so aes-fhe_amd/build/libaesfhe.so}" --scale-bits 40 --batch ${BATCH:-16} --phases
