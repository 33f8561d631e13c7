"""Single-pair solve launched eagerly (what hsflow_flow does between its
upload and download) against the same solve replayed as a hipGraph, and the
host call beside them:
    python scripts/eager_vs_graph.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import hsflow  # noqa: E402


def timed(fn, n):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    best = []
    for _ in range(3):
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        best.append((time.perf_counter() - t) / n * 1e3)
    return round(min(best), 4), round(float(np.median(best)), 4)


for rows, cols, iters in ((1080, 1920, 300), (2160, 3840, 500)):
    a, b = hsflow.synth_pair(1000, rows, cols)
    a8, b8 = a.astype(np.uint8), b.astype(np.uint8)
    I0, I1 = torch.from_numpy(a8)[None].cuda(), torch.from_numpy(b8)[None].cuda()
    u, v = torch.empty(1, rows, cols, device="cuda"), torch.empty(1, rows, cols, device="cuda")
    ws = hsflow.alloc_workspace(rows, cols, 1)
    s = torch.cuda.Stream()
    res = {"shape": f"{cols}x{rows}", "iters": iters}
    # warm the clocks
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        while time.perf_counter() - t0 < 0.2:
            hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws, s)
    torch.cuda.synchronize()

    def eager():
        with torch.cuda.stream(s):
            hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws, s)
    res["eager_ms_best_median"] = timed(eager, 20)
    g = torch.cuda.CUDAGraph()
    with hsflow.max_streams_as(2), torch.cuda.graph(g, capture_error_mode="thread_local"):
        hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws, torch.cuda.current_stream())
    res["graph_ms_best_median"] = timed(g.replay, 20)

    # one eager solve, synchronised per call (the host call's pattern)
    def eager_sync():
        eager()
        s.synchronize()
    res["eager_sync_ms_best_median"] = timed(eager_sync, 20)

    def graph_sync():
        g.replay()
        torch.cuda.current_stream().synchronize()
    res["graph_sync_ms_best_median"] = timed(graph_sync, 20)
    ctx = hsflow.Context(0)
    for dt in (np.float64, np.float32):
        ou, ov = np.empty((rows, cols), dt), np.empty((rows, cols), dt)
        res[f"host_call_{np.dtype(dt).name}_ms_best_median"] = timed(
            lambda: ctx.flow(a8, b8, 5, iters, 1.0, out_dtype=dt, out=(ou, ov)), 15)
    ctx.close()
    print(json.dumps(res), flush=True)
