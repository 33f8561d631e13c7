"""The bench times 20 graph-replayed 1080p x 8 solves after a 0.15 s
pre-warm.  What does the same solve cost under sustained load?  Replays
back to back for 3 s; the mean ms per solve in each 100 ms window, and
the shader clock read around it (rocm-smi is not needed: s_memtime /
s_memrealtime via a one-wave kernel is overkill -- the solve time itself
is the measure).  python scripts/sustained_probe.py"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import hsflow  # noqa: E402

batch, rows, cols, iters = 8, 1080, 1920, 300
ps = [hsflow.synth_pair(1000 + i, rows, cols) for i in range(batch)]
I0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
I1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
u = torch.empty((batch, rows, cols), dtype=torch.float32, device="cuda")
v = torch.empty_like(u)
ws = hsflow.alloc_workspace(rows, cols, batch)
cap = torch.cuda.Stream()
cap.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(cap):
    hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws, cap)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with hsflow.max_streams_as(2), torch.cuda.graph(g, capture_error_mode="thread_local"):
    hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws, torch.cuda.current_stream())
torch.cuda.synchronize()
windows = []
t_start = time.perf_counter()
while time.perf_counter() - t_start < 3.0:
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 0.1:
        for _ in range(4):
            g.replay()
        torch.cuda.synchronize()
        n += 4
    windows.append(round((time.perf_counter() - t0) / n * 1e3, 3))
print("RESULT " + json.dumps({"ms_per_solve_per_100ms_window": windows}), flush=True)
