# Same-box A/B over library builds x environment settings (bench.py lines).
# usage: LIBS="ab/a.so ab/b.so" CFGS="HSFLOW_JACOBI=3,HSFLOW_K3_WAVES=2 ..." WLS=1080p bash scripts/lib_env_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in ${REPS:-1}; do
  for L in $LIBS; do
    for C in $CFGS; do
      for WL in ${WLS:-1080p}; do
        env HSFLOW_LIB=$PWD/$L ${C//,/ } timeout -k 10 200 python bench.py --workload $WL --no-cpu-baseline --roofline-reps 1 $EXTRA > gpurun_out/ab.json || exit $?
        python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$L $C $WL', d['value'], 'launch_ms', d['roofline']['avg_launch_ms'])"
      done
    done
  done
done
