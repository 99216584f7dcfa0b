#!/bin/bash
# poly2_int S-box kernel (k_poly2_int_s): parity tests of the S-box kernels, then the bench round
# with the specialised kernel (AESFHE_POLY2_S=1) and the general one (=0), alternated A/B/A/B.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-p2s}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_client_path.py tests/test_aes_rows.py -x -q -m gpu -k "poly2 or sliced or sub_bytes or client or device" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
B="python3 bench.py --steps 3 --warmup 1 --no-configs --no-harness --client-batch 0 --aes10-batch 0 --no-cpu-baseline --config5 off"
n=0
for arm in 1 0 1; do
  n=$((n+1))
  AESFHE_POLY2_S=$arm timeout -k 10 300 $B > gpurun_out/${TAG}_bench_${n}_s$arm.json 2> gpurun_out/${TAG}_bench_${n}_s$arm.err || { tail -20 gpurun_out/${TAG}_bench_${n}_s$arm.err; exit 1; }
  python3 tools/brief.py gpurun_out/${TAG}_bench_${n}_s$arm.json "s=$arm"
done
