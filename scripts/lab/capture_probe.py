"""Single 1080p pair: the geom_probe graph (captured on a side stream, event
timing) against the bench's resident_leg graph (captured on the current
stream, perf_counter timing), in one process.  python scripts/lab/capture_probe.py"""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import numpy as np
import hsflow
import torch

rows, cols, w, iters = 1080, 1920, 5, 300
dev = torch.device("cuda", 0)
a, b = hsflow.synth_pair(1000, rows, cols)
I0 = torch.from_numpy(np.stack([a])).to(dev)
I1 = torch.from_numpy(np.stack([b])).to(dev)
u = torch.empty((1, rows, cols), dtype=torch.float32, device=dev)
v = torch.empty_like(u)
ws = hsflow.alloc_workspace(rows, cols, 1, dev)


def bench_style():
    stream = torch.cuda.current_stream(dev)
    cap = torch.cuda.Stream(dev)
    cap.wait_stream(stream)
    with torch.cuda.stream(cap):
        hsflow.flow_device(I0, I1, w, iters, 1.0, u, v, ws, cap)
    stream.wait_stream(cap)
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        hsflow.flow_device(I0, I1, w, iters, 1.0, u, v, ws, torch.cuda.current_stream(dev))
    torch.cuda.synchronize(dev)
    return g


def lab_style():
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        hsflow.flow_device(I0, I1, w, iters, 1.0, u, v, ws, s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        hsflow.flow_device(I0, I1, w, iters, 1.0, u, v, ws, s)
    return g


for name, mk in (("bench", bench_style), ("lab", lab_style), ("bench", bench_style), ("lab", lab_style)):
    g = mk()
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        g.replay()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    for _ in range(20):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / 20 * 1e3
    print(name, "event ms", round(e0.elapsed_time(e1) / 20, 4), "wall ms", round(wall, 4), flush=True)
