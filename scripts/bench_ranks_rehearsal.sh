# Rehearse bench.py's N > 1 path (graph capture, then process group, barrier,
# max-over-ranks timing, the config-4 stream and config-5 bands legs, one JSON
# line) with 2 ranks sharing the box's one GPU over gloo.  Not a scaling
# measurement: both ranks share a device.  The legs without communication
# are skipped (the default run covers them at N = 1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
HSFLOW_BENCH_BACKEND=gloo HSFLOW_BENCH_DEVICE=0 timeout -k 10 300 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline \
  --no-secondary --no-w3 --no-8k --no-single --no-e2e --no-host-api \
  > gpurun_out/ranks2.out 2> gpurun_out/ranks2.err
rc=$?
grep '^{' gpurun_out/ranks2.out
tail -3 gpurun_out/ranks2.err
exit $rc
