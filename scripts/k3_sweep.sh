# K3 geometry sweep: waves per strip (HSFLOW_K3_WAVES) x segment rows (HSFLOW_SEG)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
WL=${WL:-1080p}
HSFLOW_JACOBI=2 timeout -k 10 200 python bench.py --workload $WL --no-cpu-baseline --roofline-reps 1 $EXTRA > gpurun_out/sw.json || exit $?
python -c "import json; d=json.load(open('gpurun_out/sw.json')); print('K2 $WL', d['value'], 'launch_ms', d['roofline']['avg_launch_ms'])"
for S in ${SS:-3 2 6}; do
  for G in ${SEGS:-0 60 216 1080}; do
    HSFLOW_JACOBI=3 HSFLOW_K3_WAVES=$S HSFLOW_SEG=$G timeout -k 10 200 python bench.py --workload $WL --no-cpu-baseline --roofline-reps 1 $EXTRA > gpurun_out/sw.json || exit $?
    python -c "import json; d=json.load(open('gpurun_out/sw.json')); print('K3 $WL S $S seg $G', d['value'], 'launch_ms', d['roofline']['avg_launch_ms'])"
  done
done
