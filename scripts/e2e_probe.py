"""Where the end-to-end leg's time goes (bench.py e2e_leg): the same
double-buffered pipeline with copies switched off one at a time."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import hsflow  # noqa: E402

dev = torch.device("cuda", 0)
rows, cols, iters, batch = 1080, 1920, 300, 8
host_in = []
for k in range(2):
    ps = [hsflow.synth_pair(1000 + 8 * k + i, rows, cols, dtype=np.uint8) for i in range(batch)]
    host_in.append((torch.from_numpy(np.stack([p[0] for p in ps])).pin_memory(),
                    torch.from_numpy(np.stack([p[1] for p in ps])).pin_memory()))
shp = (batch, rows, cols)
d_in = [(torch.empty(shp, dtype=torch.uint8, device=dev), torch.empty(shp, dtype=torch.uint8, device=dev)) for _ in range(2)]
d_out = [(torch.empty(shp, device=dev), torch.empty(shp, device=dev)) for _ in range(2)]
h_out = [(torch.empty(shp).pin_memory(), torch.empty(shp).pin_memory()) for _ in range(2)]
ws = [hsflow.alloc_workspace(rows, cols, batch, dev) for _ in range(2)]
s_h2d, s_cmp, s_d2h = (torch.cuda.Stream(dev) for _ in range(3))
ev = {k: [torch.cuda.Event() for _ in range(2)] for k in ("in", "done", "in_free", "out_free")}


# each slot's solve as one hipGraph, as bench.e2e_leg replays it
graphs = []
cur = torch.cuda.current_stream(dev)
for sl in range(2):
    cap = torch.cuda.Stream(dev)
    cap.wait_stream(cur)
    with torch.cuda.stream(cap):
        hsflow.flow_device(d_in[sl][0], d_in[sl][1], 5, iters, 1.0, d_out[sl][0], d_out[sl][1],
                           ws[sl], cap)
    cur.wait_stream(cap)
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with hsflow.max_streams_as(2), torch.cuda.graph(g, capture_error_mode="thread_local"):
        hsflow.flow_device(d_in[sl][0], d_in[sl][1], 5, iters, 1.0, d_out[sl][0], d_out[sl][1],
                           ws[sl], torch.cuda.current_stream(dev))
    graphs.append(g)
torch.cuda.synchronize(dev)


def run(n, h2d=True, d2h=True, solve=True, kd2h=False):
    for k in range(n):
        sl = k % 2
        a, b = host_in[k % 2]
        with torch.cuda.stream(s_h2d):
            if k >= 2:
                s_h2d.wait_event(ev["in_free"][sl])
            if h2d:
                d_in[sl][0].copy_(a, non_blocking=True)
                d_in[sl][1].copy_(b, non_blocking=True)
            ev["in"][sl].record(s_h2d)
        with torch.cuda.stream(s_cmp):
            s_cmp.wait_event(ev["in"][sl])
            if k >= 2:
                s_cmp.wait_event(ev["out_free"][sl])
            if solve:
                graphs[sl].replay()
            ev["in_free"][sl].record(s_cmp)
            ev["done"][sl].record(s_cmp)
        with torch.cuda.stream(s_d2h):
            s_d2h.wait_event(ev["done"][sl])
            if d2h and kd2h:
                hsflow.download_device(h_out[sl][0], d_out[sl][0], s_d2h)
                hsflow.download_device(h_out[sl][1], d_out[sl][1], s_d2h)
            elif d2h:
                h_out[sl][0].copy_(d_out[sl][0], non_blocking=True)
                h_out[sl][1].copy_(d_out[sl][1], non_blocking=True)
            ev["out_free"][sl].record(s_d2h)
    torch.cuda.synchronize(dev)


for name, kw in (("full", {}), ("no_d2h", {"d2h": False}), ("no_h2d", {"h2d": False}),
                 ("solve_only", {"h2d": False, "d2h": False}), ("copies_only", {"solve": False}),
                 ("full", {}), ("full_kernel_d2h", {"kd2h": True}),
                 ("copies_only_kernel_d2h", {"solve": False, "kd2h": True}),
                 ("full_kernel_d2h", {"kd2h": True})):
    run(2, **kw)
    t = time.perf_counter()
    run(8, **kw)
    dt = (time.perf_counter() - t) / 8
    ok = bool(torch.equal(h_out[0][0], d_out[0][0].cpu()))
    print(json.dumps({"case": name, "last_batch_downloaded": ok, "ms_per_batch": round(dt * 1e3, 3),
                      "pairs_per_s": round(batch / dt, 1)}), flush=True)
