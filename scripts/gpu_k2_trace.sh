# K2 per-workgroup phase timeline (development trace build), default streams
# and single stream.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export HSFLOW_LIB=$PWD/cpp-optical-flow_amd/libhsflow_dev_trace.so HSFLOW_DEV_TRACE_ON=1
timeout -k 10 180 python scripts/k2_trace.py --out gpurun_out/k2_trace_default.json --raw gpurun_out/k2raw_2s > gpurun_out/k2_trace.log 2>&1 || { tail -20 gpurun_out/k2_trace.log; exit 1; }
timeout -k 10 180 python scripts/k2_trace.py --streams 1 --out gpurun_out/k2_trace_1s.json --raw gpurun_out/k2raw_1s >> gpurun_out/k2_trace.log 2>&1 || { tail -20 gpurun_out/k2_trace.log; exit 1; }
cat gpurun_out/k2_trace.log
