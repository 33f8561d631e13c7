set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc -> stop"; exit $rc; fi
timeout -k 10 300 python scripts/sweep.py --kbs 1,2,4,8 --workloads 1080p:8,4k:2,1080p:1 > gpurun_out/sweep.log 2>&1 || exit $?
cat gpurun_out/sweep.log | grep '^{'
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || exit $?
grep '^{' gpurun_out/bench.log
