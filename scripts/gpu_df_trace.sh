# Per-tile phase trace of the dataflow K2 (development trace build), 1080p x 8.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export HSFLOW_LIB=$PWD/cpp-optical-flow_amd/libhsflow_dev_dftrace.so HSFLOW_DEV_TRACE_ON=1
timeout -k 10 180 python scripts/k2_trace.py --workloads 1080p --out gpurun_out/df_trace.json --raw gpurun_out/dfraw > gpurun_out/df_trace.log 2>&1 || { tail -20 gpurun_out/df_trace.log; exit 1; }
cat gpurun_out/df_trace.log
