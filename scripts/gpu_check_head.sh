# GPU test suite + default bench line of the current build (no ubench).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench_default.err; cat gpurun_out/bench_default.json; exit 1; }
cat gpurun_out/bench_default.json
