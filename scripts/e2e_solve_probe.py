"""Is the e2e leg's solve slower than the resident one, and why?  Graph-
replayed 1080p x 8 solves (batch split over the side streams, after a
0.15 s pre-warm): f32 frames (the resident leg) and u8 frames (the e2e
leg), then the u8 solve again while a D2H of 133 MB runs beside each replay
(the e2e pipeline's overlap).  python scripts/e2e_solve_probe.py"""
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
F0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
F1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
out = {}
for name, (I0, I1) in (("f32", (F0, F1)), ("u8", (F0.to(torch.uint8), F1.to(torch.uint8)))):
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
    t = time.perf_counter()
    n = 0
    while time.perf_counter() - t < 0.15:
        g.replay()
        n += 1
        if n % 4 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    out[name] = round(e0.elapsed_time(e1) / 20, 4)
    if name == "u8":
        hu = torch.empty((batch, rows, cols), dtype=torch.float32).pin_memory()
        hv = torch.empty_like(hu).pin_memory()
        s_d = torch.cuda.Stream()
        ev = [torch.cuda.Event() for _ in range(20)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(20):
            g.replay()
            ev[k].record()
            s_d.wait_event(ev[k])
            hsflow.download_device(hu, u, s_d)
            hsflow.download_device(hv, v, s_d)
        torch.cuda.synchronize()
        out["u8_with_d2h_beside"] = round((time.perf_counter() - t0) / 20 * 1e3, 4)
print("RESULT " + json.dumps(out), flush=True)
