set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_strips.py tests/test_bench_golden.py tests/test_input_path.py tests/test_output_path.py -x -q --timeout 120 --timeout-method thread > gpurun_out/k1_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/k1_tests.log; exit 1; }
tail -2 gpurun_out/k1_tests.log
timeout -k 10 300 python -u scripts/lab/k4_variants.py probe prev cur > gpurun_out/k1_ab.txt 2>&1 && timeout -k 10 300 python -u scripts/lab/k4_variants.py probe cur prev >> gpurun_out/k1_ab.txt 2>&1
cat gpurun_out/k1_ab.txt
