#!/bin/bash
# Rehearse bench.py's N > 1 path (graph capture, then process group, barrier,
# max-over-ranks timing, the config-4 stream and config-5 bands legs, one JSON
# line) with N ranks (default 2; 4 gives the 2 x 2 block grid, corners
# included) sharing the box's one GPU over gloo.  Not a scaling measurement:
# the ranks share a device.  The legs without communication are skipped (the
# default run covers them at N = 1).
#   bash scripts/bench_ranks_rehearsal.sh [N]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
N=${1:-2}
HSFLOW_BENCH_BACKEND=gloo HSFLOW_BENCH_DEVICE=0 timeout -k 10 400 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
  --master-port $((29510 + N)) bench.py --gpus "$N" --steps 3 --warmup 1 --no-cpu-baseline \
  --no-secondary --no-w3 --no-8k --no-single --no-e2e --no-host-api \
  > gpurun_out/ranks$N.out 2> gpurun_out/ranks$N.err
rc=$?
grep '^{' gpurun_out/ranks$N.out
tail -3 gpurun_out/ranks$N.err
exit $rc
