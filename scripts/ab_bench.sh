# Same-box A/B of two libhsflow builds through bench.py (alternating runs).
# usage: LIBS="ab/libhsflow_prev.so cpp-optical-flow_amd/libhsflow.so" bash scripts/ab_bench.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for L in $LIBS; do
    for WL in ${WLS:-1080p 4k}; do
      HSFLOW_LIB=$PWD/$L timeout -k 10 200 python bench.py --workload $WL --no-cpu-baseline --roofline-reps 1 $EXTRA > gpurun_out/ab.json || exit $?
      python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$L', '$WL', d['value'], 'kb', d['config']['iters_per_launch'], 'launch_ms', d['roofline']['avg_launch_ms'])"
    done
  done
done
