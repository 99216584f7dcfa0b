#!/bin/bash
# Round 5 debugging: the bit-exact parity file with the matrix-core base conversions, then the
# ten-round test with the VALU ones and with the matrix-core ones (serialised launches).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-dbg}
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
timeout -k 10 400 python -u -X faulthandler -m pytest tests/test_gpu_parity.py -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_parity.log 2>&1; rc=$?
tail -25 gpurun_out/${TAG}_parity.log; fatal $rc parity
AESFHE_BCONV_VALU=1 timeout -k 10 300 python -u -X faulthandler -m pytest tests/test_aes128_full.py -x -q -m gpu -k full_params --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_aes_valu.log 2>&1; rc=$?
tail -5 gpurun_out/${TAG}_aes_valu.log; fatal $rc aes_valu
AMD_SERIALIZE_KERNEL=3 AMD_LOG_LEVEL=1 timeout -k 10 300 python -u -X faulthandler -m pytest tests/test_aes128_full.py -x -q -m gpu -k full_params --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_aes_mfma.log 2>&1; rc=$?
tail -30 gpurun_out/${TAG}_aes_mfma.log; fatal $rc aes_mfma
