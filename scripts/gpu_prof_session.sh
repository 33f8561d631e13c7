# Config-4 GPU tests (serial + overlapped schedules), then the rocprofv3
# evidence of the default bench command (scripts/gpu_prof_bench.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_bench_golden.py -m gpu -k config4 -x -v --timeout 200 --timeout-method thread > gpurun_out/c4.log 2>&1 || { echo "c4 failed"; tail -30 gpurun_out/c4.log; exit 1; }
tail -4 gpurun_out/c4.log
bash scripts/gpu_prof_bench.sh
