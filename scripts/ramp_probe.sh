# Bench value vs run length, with and without the 2-stream batch split.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for ST in 2 1; do
  for sw in "3 1" "3 5" "10 2"; do
    set -- $sw
    HSFLOW_STREAMS=$ST timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-cpu-baseline > gpurun_out/ramp.json || exit $?
    python -c "import json; d=json.load(open('gpurun_out/ramp.json')); print('streams $ST steps/warmup $1/$2', d['value'], d['ms_per_step'])"
  done
done
