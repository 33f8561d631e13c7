# Dataflow K2 development check: bit-identity vs per-pass launches, then a
# same-box timing A/B against the per-pass development library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export HSFLOW_LIB=$PWD/cpp-optical-flow_amd/libhsflow_dev_df.so
timeout -k 10 240 python -u scripts/df_check.py > gpurun_out/df_check.log 2>&1 || { echo "df_check rc=$?"; tail -30 gpurun_out/df_check.log; exit 1; }
cat gpurun_out/df_check.log
unset HSFLOW_LIB
rm -f gpurun_out/devab.log
ROUNDS="1 2" bash scripts/gpu_devab.sh tpf df || exit $?
