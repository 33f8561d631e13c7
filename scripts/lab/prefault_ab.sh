set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_output_path.py tests/test_input_path.py tests/test_cv_adapter.py tests/test_gpu_parity.py tests/test_pyramid.py tests/test_frame_parallel.py -x -q --timeout 120 --timeout-method thread > gpurun_out/prefault_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/prefault_tests.log; exit 1; }
tail -2 gpurun_out/prefault_tests.log
timeout -k 10 500 python -u scripts/lab/hostio_variants.py probe prev cur > gpurun_out/prefault_ab.txt 2>&1
tail -1 gpurun_out/prefault_ab.txt
