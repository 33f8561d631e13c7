# Memory-only / compute-only / full K2 launch times (HSFLOW_ABLATE 1 / 2 / 0)
# for a batch that streams from HBM and one that stays in the Infinity Cache.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for B in ${BATCHES:-8 1}; do
  for A in 0 1 2; do
    for PF in ${PFS:-0}; do
      HSFLOW_PF=$PF HSFLOW_STREAMS=1 HSFLOW_ABLATE=$A timeout -k 10 200 python bench.py --workload ${WL:-1080p} --batch $B --steps 3 --warmup 1 --no-cpu-baseline --roofline-reps 2 > gpurun_out/sp.json || exit $?
      python -c "import json; d=json.load(open('gpurun_out/sp.json')); r=d['roofline']; print('batch $B ablate $A pf $PF', 'launch_us %.1f' % (1e3*r['avg_launch_ms']), 'us_per_Mpx %.2f' % (1e3*r['avg_launch_ms']/($B*${PX:-2.0736})))"
    done
  done
done
