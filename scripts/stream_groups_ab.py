"""Same-box A/B of the config-4 stream leg at N = 1: 64 pairs solved in one
call vs in groups of 8 (bench.stream_leg's grouping), alternated twice.
    python scripts/stream_groups_ab.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cpp-optical-flow_amd")]
import torch  # noqa: E402
import frame_parallel as fp  # noqa: E402
import hsflow  # noqa: E402

dev = torch.device("cuda", 0)
rows, cols, iters, n = 1080, 1920, 300, 64
stream = [tuple(torch.from_numpy(a).to(dev) for a in hsflow.synth_pair(1000 + j, rows, cols))
          for j in range(n)]
wss = {}


def solve_batch(I0, I1):
    b = I0.shape[0]
    if b not in wss:
        wss[b] = hsflow.alloc_workspace(rows, cols, b, dev)
    return hsflow.flow_device(I0, I1, 5, iters, 1.0, workspace=wss[b])


for chunks in (1, 8, 1, 8):
    fp.run_stream_pipelined(stream, n, (rows, cols), torch.float32, solve_batch, dev, 0, 1,
                            chunks=chunks)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        out = fp.run_stream_pipelined(stream, n, (rows, cols), torch.float32, solve_batch, dev,
                                      0, 1, chunks=chunks)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 3
    print(json.dumps({"groups": chunks, "pairs_per_s": round(n / dt, 1),
                      "Mpix_iter_per_s": round(n * rows * cols * iters / dt / 1e6)}), flush=True)
