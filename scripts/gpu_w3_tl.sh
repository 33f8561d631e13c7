# Window 3: tall T-in-LDS slabs (11 rows, now with the T read one row ahead)
# vs the all-register 10-row slabs, probe build, same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; rm -f gpurun_out/w3tl.log
export HSFLOW_LIB=$PWD/cpp-optical-flow_amd/libhsflow_probe.so
for round in 1 2; do
  for TL in 0 1; do
    HSFLOW_K2_TL=$TL timeout -k 10 120 python scripts/solve_ab.py --tag tl$TL --window ${W:-3} --reps 10 >> gpurun_out/w3tl.log 2>&1 || exit $?
  done
done
grep '^{' gpurun_out/w3tl.log
