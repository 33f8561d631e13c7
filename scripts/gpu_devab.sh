# Same-box A/B of development libraries (scripts/build_dev.sh): each tag's
# bench-shaped solve, alternated twice.  usage: gpu_devab.sh TAG1 TAG2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for round in ${ROUNDS:-1 2}; do
  for T in "$@"; do
    HSFLOW_LIB=$PWD/cpp-optical-flow_amd/libhsflow_dev_$T.so timeout -k 10 120 \
      python scripts/solve_ab.py --tag $T --reps 10 >> gpurun_out/devab.log 2>&1 || exit $?
  done
done
grep '^{' gpurun_out/devab.log
