# rocprofv3 passes over bench.py for one workload: kernel trace + stats, then
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md
# §rocprofv3: FETCH_SIZE and WRITE_SIZE do not fit one pass).
# HSFLOW_STREAMS=1 keeps K2 dispatches single-stream so the per-dispatch
# average matches bench.py's roofline timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp HSFLOW_STREAMS=1
WL=${WL:-1080p}; P=gpurun_out/${PROF_TAG:-prof}_$WL; mkdir -p $P
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --roofline-reps 2 --workload $WL"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 $B > $P/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run --output-format csv -- python3 $B > $P/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $P/write -o run --output-format csv -- python3 $B > $P/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $P/sq -o run --output-format csv -- python3 $B > $P/sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT -d $P/tcc -o run --output-format csv -- python3 $B > $P/tcc.log 2>&1 || exit $?
grep '^{' $P/trace.log | tail -1
