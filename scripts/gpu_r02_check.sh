# Round-2 check: VALU ubench (cycles via s_memtime), GPU test suite, default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 60 ./scripts/ubench/valu_tput > gpurun_out/r02_valu_tput.txt 2>&1 || { echo "ubench failed"; cat gpurun_out/r02_valu_tput.txt; exit 1; }
cat gpurun_out/r02_valu_tput.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r02_pytest.log; exit 1; }
tail -3 gpurun_out/r02_pytest.log
timeout -k 10 400 python bench.py > gpurun_out/r02_bench_default.json 2> gpurun_out/r02_bench_default.err || { echo "bench rc=$?"; tail -20 gpurun_out/r02_bench_default.err; cat gpurun_out/r02_bench_default.json; exit 1; }
cat gpurun_out/r02_bench_default.json
