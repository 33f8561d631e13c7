set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_strips.py tests/test_gpu_parity.py tests/test_bench_golden.py tests/test_pyramid.py tests/test_row_bands.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wg2_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/wg2_tests.log; exit 1; }
tail -2 gpurun_out/wg2_tests.log
timeout -k 10 300 python -u scripts/lab/k4_variants.py probe prev wg2 > gpurun_out/wg2_ab.txt 2>&1 && timeout -k 10 300 python -u scripts/lab/k4_variants.py probe wg2 prev >> gpurun_out/wg2_ab.txt 2>&1
grep "^{" gpurun_out/wg2_ab.txt
