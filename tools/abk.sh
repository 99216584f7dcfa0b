set -o pipefail
# alternated A/B/A/B kernel profiles: A = build/libaesfhe_old.so, B = build/libaesfhe.so; extra args go to bench.py
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abk
for v in A B A2 B2; do
  lib=$PWD/aes-fhe_amd/build/libaesfhe_old.so; case $v in B*) lib=$PWD/aes-fhe_amd/build/libaesfhe.so;; esac
  AESFHE_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abk/prof_$v -o k -- python bench.py --no-cpu-baseline --no-configs --aes10-batch 0 --steps 1 --warmup 1 "$@" > gpurun_out/abk/prof_$v.log 2>&1 || exit 1
  rm -f gpurun_out/abk/prof_$v/*_kernel_trace.csv
  echo "$v done"
done
