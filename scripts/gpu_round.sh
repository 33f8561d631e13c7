#!/bin/bash
# Round evidence of the tree as it is (on the GPU box): the GPU test suite,
# smoke(), the default bench line, then a kernel trace of the bench's primary
# leg checked against its ms_per_step (scripts/trace_fit.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
t0=$SECONDS
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err \
    || { echo "bench rc=$?"; tail -20 gpurun_out/bench_default.err; cat gpurun_out/bench_default.json; exit 1; }
echo "bench wall seconds: $((SECONDS - t0))" | tee gpurun_out/bench_wall.txt
cat gpurun_out/bench_default.json
[ "$1" = "--trace" ] || exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bench_trace -o run --output-format csv -- \
    python3 bench.py --no-secondary --no-w3 --no-8k --no-single --no-e2e --no-stream --no-cpu-baseline --no-bands --no-host-api \
    > gpurun_out/bench_trace.json 2> gpurun_out/bench_trace.err || { echo "trace failed"; exit 1; }
python3 scripts/trace_fit.py gpurun_out/bench_trace gpurun_out/bench_trace.json
