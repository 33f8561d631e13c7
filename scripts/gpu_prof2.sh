set -o pipefail
cd "$GRAFT_REPO_ROOT"; P=gpurun_out/${PROF_TAG:-prof}; mkdir -p $P; export TMPDIR=/tmp
rocprofv3 -L > $P/counters_list.txt 2>&1 || true
B="scripts/sweep.py --kbs 4 --workloads 1080p:8 --rounds 2 --iters 40"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES -d $P/sq -o run --output-format csv -- python3 $B > $P/sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT -d $P/sq2 -o run --output-format csv -- python3 $B > $P/sq2.log 2>&1 || true
HSFLOW_ABLATE=2 timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $P/sqabl -o run --output-format csv -- python3 $B > $P/sqabl.log 2>&1 || exit $?
echo done
