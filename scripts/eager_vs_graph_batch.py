"""Batched solves (the bench's headline and 4K shapes) launched eagerly
against the same solve replayed as a hipGraph, back to back, alternated in
rounds on one box:
    python scripts/eager_vs_graph_batch.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import hsflow  # noqa: E402


def run(fn, n):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


for rows, cols, iters, batch in ((1080, 1920, 300, 8), (2160, 3840, 500, 2), (1080, 1920, 300, 1)):
    pairs = [hsflow.synth_pair(1000 + k, rows, cols) for k in range(batch)]
    I0 = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    I1 = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    u, v = torch.empty_like(I0), torch.empty_like(I0)
    ws = hsflow.alloc_workspace(rows, cols, batch)
    s = torch.cuda.Stream()

    def eager():
        with torch.cuda.stream(s):
            hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws, s)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        eager()
    torch.cuda.synchronize()
    ref = u.clone()
    g = torch.cuda.CUDAGraph()
    with hsflow.max_streams_as(2), torch.cuda.graph(g, capture_error_mode="thread_local"):
        hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws, torch.cuda.current_stream())
    n = max(5, int(40 / batch))
    e, gr = [], []
    for r in range(6):
        e.append(run(eager, n))
        gr.append(run(g.replay, n))
    eq = bool(torch.equal(u, ref))
    mpix = rows * cols * iters * batch / 1e6
    res = {"shape": f"{cols}x{rows}", "batch": batch, "iters": iters,
           "eager_ms": [round(x, 4) for x in e], "graph_ms": [round(x, 4) for x in gr],
           "eager_median_M": round(mpix / np.median(e) * 1e3 / 1e6, 4),
           "graph_median_M": round(mpix / np.median(gr) * 1e3 / 1e6, 4), "bits_equal": eq}
    print(json.dumps(res), flush=True)
    del g
