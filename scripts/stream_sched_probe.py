"""Diagnostic: the config-4 stream schedules (serial run_stream vs the
overlapped run_stream_pipelined) with 2 ranks over gloo sharing the box's
one GPU, CUDA tensors as in bench.py's rehearsal.  Prints per-schedule time.
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        scripts/stream_sched_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import frame_parallel as fp  # noqa: E402
import hsflow  # noqa: E402

dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
rows, cols, iters, n = 1080, 1920, 30, int(os.environ.get("PAIRS", "8"))
stream = None
if rank == 0:
    stream = [tuple(torch.from_numpy(a).to(dev) for a in hsflow.synth_pair(1000 + j, rows, cols))
              for j in range(n)]


def solve_batch(I0, I1):
    return hsflow.flow_device(I0, I1, 5, iters, 1.0)


def solve_one(I0, I1):
    u, v = hsflow.flow_device(I0[None], I1[None], 5, iters, 1.0)
    return u[0], v[0]


for name, fn in (("serial", lambda: fp.run_stream(stream, n, (rows, cols), torch.float32,
                                                  solve_one, dev, rank, world)),
                 ("pipelined", lambda: fp.run_stream_pipelined(stream, n, (rows, cols),
                                                               torch.float32, solve_batch, dev,
                                                               rank, world, chunks=2))):
    for rep in range(2):
        dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        dist.barrier()
        if rank == 0:
            print(f"{name} rep {rep}: {time.perf_counter() - t:.3f} s", flush=True)
dist.destroy_process_group()
