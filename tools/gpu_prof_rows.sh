set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rows -o rows -- python3 tools/round_stages.py rows 8 > gpurun_out/prof_rows.log 2>&1
rc=$?; tail -8 gpurun_out/prof_rows.log; find gpurun_out/prof_rows -name "*stats*"; exit $rc
