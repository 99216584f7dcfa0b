set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -k "power_basis" --timeout 300 --timeout-method thread > gpurun_out/pytest_pb.log 2>&1 \
 && echo "tests ok" \
 && timeout -k 10 200 python3 tools/config_prof.py --legs 2 --reps 2 > gpurun_out/c2_pb.json 2> gpurun_out/c2_pb.err \
 && echo "legs ok" \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c2prof_pb -o c2 -- python3 tools/config_prof.py --legs 2 > gpurun_out/c2prof_pb.log 2>&1 \
 && echo "prof ok"
rc=$?
tail -5 gpurun_out/pytest_pb.log; cat gpurun_out/c2_pb.json
exit $rc
