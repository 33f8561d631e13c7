set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/e2e_trace
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/e2e_trace -o run --output-format csv -- python3 scripts/e2e_probe.py > gpurun_out/e2e_trace/log.txt 2>&1
rc=$?; grep '^{' gpurun_out/e2e_trace/log.txt; ls gpurun_out/e2e_trace/*/ 2>/dev/null | head; exit $rc
