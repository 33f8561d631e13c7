set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof2; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc -> stop"; exit $rc; fi
timeout -k 10 300 python scripts/sweep.py --kbs 2,4,8 --workloads 1080p:8,4k:2,1080p:1 > gpurun_out/sweep.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep.log
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --roofline-reps 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof2/fetch -o run --output-format csv -- python3 $B > gpurun_out/prof2/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof2/tcc -o run --output-format csv -- python3 $B > gpurun_out/prof2/tcc.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || exit $?
grep '^{' gpurun_out/bench.log
