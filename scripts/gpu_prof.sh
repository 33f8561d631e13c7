set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --roofline-reps 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python3 $B > gpurun_out/prof/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o run --output-format csv -- python3 $B > gpurun_out/prof/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o run --output-format csv -- python3 $B > gpurun_out/prof/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/prof/sq -o run --output-format csv -- python3 $B > gpurun_out/prof/sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof/tcc -o run --output-format csv -- python3 $B > gpurun_out/prof/tcc.log 2>&1 || exit $?
timeout -k 10 300 python scripts/sweep.py --kbs 2,4,8 --workloads 1080p:8,4k:2,1080p:1 > gpurun_out/sweep.log 2>&1 || exit $?
find gpurun_out/prof -name "*.csv" | head -20
