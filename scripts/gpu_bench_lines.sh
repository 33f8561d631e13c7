# Bench lines of the current build (no profiling): the default run (with the
# CPU baselines), 4K, w 3 at 1080p/4K, 8K config 5, config 4 stream mode.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
B="timeout -k 10 300 python bench.py"
$B > gpurun_out/bl_default.json || exit $?
$B --workload 4k > gpurun_out/bl_4k.json || exit $?
$B --window 3 --no-cpu-baseline > gpurun_out/bl_w3.json || exit $?
$B --window 3 --workload 4k --no-cpu-baseline > gpurun_out/bl_w3_4k.json || exit $?
$B --workload 8k --no-cpu-baseline > gpurun_out/bl_8k.json || exit $?
$B --mode stream --no-cpu-baseline > gpurun_out/bl_stream.json || exit $?
for f in gpurun_out/bl_*.json; do echo "$f $(head -c 160 $f)"; done
