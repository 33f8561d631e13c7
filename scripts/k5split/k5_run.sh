set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_strips.py -x -q --timeout 120 --timeout-method thread > gpurun_out/k5_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/k5_tests.log; exit 1; }
tail -3 gpurun_out/k5_tests.log
timeout -k 10 300 python -u scripts/k4_sweep.py --kernel 4 --cases 1080p8,4k2,4k1 --windows 5 --rows-list 84 > gpurun_out/k5_sweep.txt 2>&1 &&
timeout -k 10 300 python -u scripts/k4_sweep.py --kernel 5 --cases 1080p8,4k2,4k1 --windows 5 --rows-list 60,84,108,132 >> gpurun_out/k5_sweep.txt 2>&1 &&
timeout -k 10 300 python -u scripts/k4_sweep.py --kernel 4 --cases 1080p8,4k2,4k1 --windows 5 --rows-list 84 >> gpurun_out/k5_sweep.txt 2>&1
cat gpurun_out/k5_sweep.txt
