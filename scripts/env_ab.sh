# Same-box A/B of environment settings through bench.py (alternating runs).
# usage: CFGS="HSFLOW_PF=0 HSFLOW_PF=-1" WLS="1080p 4k" bash scripts/env_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
  for C in $CFGS; do
    for WL in ${WLS:-1080p 4k}; do
      env ${C//,/ } timeout -k 10 200 python bench.py --workload $WL --no-cpu-baseline --roofline-reps 1 $EXTRA > gpurun_out/ab.json || exit $?
      python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$C', '$WL', d['value'], 'kb', d['config']['iters_per_launch'], 'launch_ms', d['roofline']['avg_launch_ms'])"
    done
  done
done
