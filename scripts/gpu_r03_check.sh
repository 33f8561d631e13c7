#!/bin/bash
# GPU regression check: the -m gpu suite, then smoke(), each under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
tag=${1:-r03}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/${tag}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids
