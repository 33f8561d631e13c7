set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head; exit $rc; }
echo "== torchrun nccl world 1 (resident)"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/dist1.log 2>&1 || { tail -20 gpurun_out/dist1.log; exit 1; }
grep '^{' gpurun_out/dist1.log
echo "== stream mode (config 4), world 1"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --mode stream --pairs 16 --steps 2 --warmup 1 > gpurun_out/stream1.log 2>&1 || { tail -20 gpurun_out/stream1.log; exit 1; }
grep '^{' gpurun_out/stream1.log
echo "== window 3"
timeout -k 10 300 python bench.py --window 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/w3.log 2>&1 || exit 1
grep '^{' gpurun_out/w3.log
