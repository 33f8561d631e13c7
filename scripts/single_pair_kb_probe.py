"""Single-pair solve time (the reference's call pattern: one getFlow per
pair) against the blocking depth, graph-replayed device solves:
    python scripts/single_pair_kb_probe.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import hsflow  # noqa: E402

for rows, cols, iters, window in ((1080, 1920, 300, 5), (720, 1280, 300, 5), (2160, 3840, 500, 5),
                                  (375, 1242, 100, 5), (1080, 1920, 300, 3)):
    a, b = hsflow.synth_pair(1000, rows, cols)
    I0, I1 = torch.from_numpy(a)[None].cuda(), torch.from_numpy(b)[None].cuda()
    u, v = torch.empty_like(I0), torch.empty_like(I0)
    ws = hsflow.alloc_workspace(rows, cols, 1)
    res = {"shape": f"{cols}x{rows}", "iters": iters, "window": window}
    ref = None
    for kb in (4, 5, 6, 8):
        hsflow.set_iters_per_launch(kb)
        if hsflow.iters_per_launch(rows, cols, 1, window) != kb:
            continue
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            hsflow.flow_device(I0, I1, window, iters, 1.0, u, v, ws, s)
        torch.cuda.synchronize()
        with hsflow.max_streams_as(2), torch.cuda.graph(g, capture_error_mode="thread_local"):
            hsflow.flow_device(I0, I1, window, iters, 1.0, u, v, ws, torch.cuda.current_stream())
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            g.replay()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / 10 * 1e3
        same = True if ref is None else bool(torch.equal(u, ref))
        ref = u.clone() if ref is None else ref
        res[f"kb{kb}_ms"] = round(ms, 3)
        res[f"kb{kb}_bits_equal"] = same
        del g
    hsflow.set_iters_per_launch(0)
    print(json.dumps(res), flush=True)
