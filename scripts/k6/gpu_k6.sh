#!/bin/bash
# K6 development round on the GPU box: its bit-identity tests, then the
# single-pair A/B against K2 (scripts/k6_probe.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_resident.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/k6_tests.log 2>&1; rc=$?
tail -25 gpurun_out/k6_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/k6_probe.py gpurun_out/k6_probe.json
