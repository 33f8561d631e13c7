# bench value vs the number of side streams a batch is split over (same box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for S in ${SPLITS:-1 2 4 8}; do
    for WL in ${WLS:-1080p 4k}; do
      HSFLOW_STREAMS=$S timeout -k 10 200 python bench.py --workload $WL --no-cpu-baseline --roofline-reps 1 $EXTRA > gpurun_out/sab.json || exit $?
      python -c "import json; d=json.load(open('gpurun_out/sab.json')); print('streams $S', '$WL', d['value'])"
    done
  done
done
