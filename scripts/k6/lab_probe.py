"""Time the K6 solve of one 1080p pair (w 5, 300 it) with a K6 lab library
(k6lab/build.sh); K2 from the same library as the same-process reference."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
import hsflow
hsflow.LIB_PATH = os.path.join(HERE, f"libhsflow_{sys.argv[1]}.so")
import torch

rows, cols, w, iters = 1080, 1920, 5, 300
kb = int(sys.argv[2]) if len(sys.argv) > 2 else 0


def timed(kernel, I0, I1, reps=30):
    hsflow.set_jacobi_kernel(kernel)
    hsflow.set_iters_per_launch(kb)
    ws = hsflow.alloc_workspace(rows, cols, 1)
    u = torch.empty(1, rows, cols, device="cuda")
    v = torch.empty_like(u)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        hsflow.flow_device(I0, I1, w, iters, 1.0, u, v, ws, s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        hsflow.flow_device(I0, I1, w, iters, 1.0, u, v, ws, s)
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        g.replay()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    hsflow.set_jacobi_kernel(0)
    return e0.elapsed_time(e1) / reps, u.clone()


a, b = hsflow.synth_pair(1000, rows, cols)
I0, I1 = torch.from_numpy(a)[None].cuda(), torch.from_numpy(b)[None].cuda()
ms2, u2 = timed(2, I0, I1)
ms6, u6 = timed(6, I0, I1)
print(f"{sys.argv[1]:10s} kb {kb}: K2 {ms2:.4f} ms  K6 {ms6:.4f} ms  same={bool(torch.equal(u2, u6))}",
      flush=True)
