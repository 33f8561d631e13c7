# Probe-build ablations of K2 (timing only; results are wrong by design):
# 0 full, 1 no iterations, 2 loads/stores out of range, 3 no barriers,
# 4 no T-plane reads.  Same box, graph-replayed bench-shaped solves.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export HSFLOW_LIB=$PWD/cpp-optical-flow_amd/libhsflow_probe.so
for A in 0 3 4 2 1 0; do
  HSFLOW_ABLATE=$A timeout -k 10 120 python scripts/solve_ab.py --tag abl$A --reps 10 >> gpurun_out/abl2.log 2>&1 || exit $?
done
cat gpurun_out/abl2.log
