# Round evidence for the current default build: rocprofv3 trace/stats and PMC
# passes (scripts/gpu_prof.sh) for 1080p and 4K, then full bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for WL in 1080p 4k; do
  WL=$WL PROF_TAG=${PROF_TAG:-final} bash scripts/gpu_prof.sh > gpurun_out/prof_$WL.out 2>&1 || { echo "prof $WL failed"; tail -5 gpurun_out/prof_$WL.out; exit 1; }
  echo "prof $WL ok"
done
B="timeout -k 10 300 python bench.py"
$B > gpurun_out/bench_default.json || exit $?
$B --workload 4k > gpurun_out/bench_4k.json || exit $?
$B --window 3 --no-cpu-baseline > gpurun_out/bench_w3.json || exit $?
$B --window 3 --workload 4k --no-cpu-baseline > gpurun_out/bench_w3_4k.json || exit $?
$B --workload 8k --no-cpu-baseline > gpurun_out/bench_8k.json || exit $?
HSFLOW_JACOBI=3 HSFLOW_STREAMS=1 $B --no-cpu-baseline > gpurun_out/bench_k3.json || exit $?
HSFLOW_JACOBI=3 HSFLOW_STREAMS=1 $B --workload 4k --no-cpu-baseline > gpurun_out/bench_k3_4k.json || exit $?
for f in gpurun_out/bench_*.json; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['config']['workload'], d['roofline']['avg_launch_ms'], d.get('cpu_baseline'))")"; done
