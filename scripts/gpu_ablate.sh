set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for A in 0 1 2; do
  HSFLOW_ABLATE=$A timeout -k 10 300 python scripts/sweep.py --kbs ${KBS:-4,8} --workloads ${WLS:-1080p:8,4k:2} > gpurun_out/abl_$A.log 2>&1 || exit $?
  echo "ablate $A"; grep '^{' gpurun_out/abl_$A.log
done
export TMPDIR=/tmp; P=gpurun_out/prof_v3; mkdir -p $P
B="scripts/sweep.py --kbs 4 --workloads 1080p:8 --rounds 2 --iters 40"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_WAVES -d $P/sq -o run --output-format csv -- python3 $B > $P/sq.log 2>&1 || exit $?
HSFLOW_ABLATE=2 timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_WAVES -d $P/sqabl -o run --output-format csv -- python3 $B > $P/sqabl.log 2>&1 || exit $?
echo done
