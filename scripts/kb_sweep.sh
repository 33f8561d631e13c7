# Same-box sweep of the blocking depth (iterations per launch) for bench.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for WL in ${WLS:-1080p 4k}; do
  for KB in ${KBS:-4 5 6 8}; do
    timeout -k 10 200 python bench.py --workload $WL --kb $KB --no-cpu-baseline --roofline-reps 1 $EXTRA > gpurun_out/kb.json || exit $?
    python -c "import json; d=json.load(open('gpurun_out/kb.json')); print('$WL kb $KB', d['value'], 'launch_ms', d['roofline']['avg_launch_ms'])"
  done
done
