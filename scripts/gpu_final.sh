# Round evidence of the current build: GPU test suite, default bench line,
# then rocprofv3 of the default bench command (scripts/gpu_prof_bench.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash scripts/gpu_check_head.sh || exit $?
bash scripts/gpu_prof_bench.sh
