set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_strips.py tests/test_gpu_parity.py tests/test_bench_golden.py -x -q --timeout 120 --timeout-method thread > gpurun_out/unpack_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/unpack_tests.log; exit 1; }
tail -2 gpurun_out/unpack_tests.log
timeout -k 10 400 python -u scripts/lab/k4_variants.py probe base oldunpack > gpurun_out/unpack_ab.txt 2>&1 && timeout -k 10 400 python -u scripts/lab/k4_variants.py probe oldunpack base >> gpurun_out/unpack_ab.txt 2>&1
cat gpurun_out/unpack_ab.txt
