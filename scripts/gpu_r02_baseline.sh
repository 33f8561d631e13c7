# Round-2 entry check: GPU parity suite and the default + 4K bench lines of the
# restored build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r02_pytest.log; exit 1; }
tail -3 gpurun_out/r02_pytest.log
timeout -k 10 300 python bench.py > gpurun_out/r02_bench_default.json || exit $?
timeout -k 10 300 python bench.py --workload 4k --no-cpu-baseline > gpurun_out/r02_bench_4k.json || exit $?
cat gpurun_out/r02_bench_default.json gpurun_out/r02_bench_4k.json
