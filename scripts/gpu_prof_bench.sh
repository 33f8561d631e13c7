# rocprofv3 of the exact default bench command (kernel trace + stats), then
# per-dispatch PMC passes (FETCH_SIZE, WRITE_SIZE and SQ counters in
# separate runs, MI355X_MICROARCH.md rocprofv3 slots), then the VALU ubench.
# Summarise with: python scripts/prof_bench.py gpurun_out/prof_bench <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
P=gpurun_out/prof_bench; mkdir -p $P
timeout -k 10 60 ./scripts/ubench/valu_tput > $P/valu_tput.txt 2>&1 || { cat $P/valu_tput.txt; exit 1; }
cat $P/valu_tput.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 bench.py > $P/trace.log 2>&1 || { tail -20 $P/trace.log; exit 1; }
grep '^{' $P/trace.log | tail -1
B="bench.py --no-cpu-baseline --no-e2e --no-stream --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run --output-format csv -- python3 $B > $P/fetch.log 2>&1 || { tail -20 $P/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $P/write -o run --output-format csv -- python3 $B > $P/write.log 2>&1 || { tail -20 $P/write.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $P/sq -o run --output-format csv -- python3 $B > $P/sq.log 2>&1 || { tail -20 $P/sq.log; exit 1; }
echo profiled
