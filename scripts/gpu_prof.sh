set -o pipefail
cd "$GRAFT_REPO_ROOT"; P=gpurun_out/${PROF_TAG:-prof}; mkdir -p $P; export TMPDIR=/tmp
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --roofline-reps 1 ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 $B > $P/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run --output-format csv -- python3 $B > $P/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $P/write -o run --output-format csv -- python3 $B > $P/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $P/sq -o run --output-format csv -- python3 $B > $P/sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU -d $P/tcc -o run --output-format csv -- python3 $B > $P/tcc.log 2>&1 || exit $?
echo done
