# Row-band GPU tests (plain and overlapped schedules) and the one-GPU
# virtual-rank probe of both schedules.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_row_bands.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/bands_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/bands_tests.log; exit 1; }
tail -3 gpurun_out/bands_tests.log
timeout -k 10 300 python -u scripts/bands_overlap_probe.py --ranks 8 --chunk 12 > gpurun_out/bands_probe.log 2>&1 || { tail -20 gpurun_out/bands_probe.log; exit 1; }
timeout -k 10 300 python -u scripts/bands_overlap_probe.py --ranks 8 --chunk 24 >> gpurun_out/bands_probe.log 2>&1 || { tail -20 gpurun_out/bands_probe.log; exit 1; }
grep '^{' gpurun_out/bands_probe.log
