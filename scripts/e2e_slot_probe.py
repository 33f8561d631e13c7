import json, os, sys, time
import numpy as np, torch
sys.path.insert(0, "cpp-optical-flow_amd")
import hsflow
batch, rows, cols, iters = 8, 1080, 1920, 300
dev = torch.device("cuda", 0)
ps = [hsflow.synth_pair(1000 + i, rows, cols, dtype=np.uint8) for i in range(batch)]
hA = torch.from_numpy(np.stack([p[0] for p in ps])).pin_memory()
hB = torch.from_numpy(np.stack([p[1] for p in ps])).pin_memory()
shp = (batch, rows, cols)
slots = 3
d_in = [(torch.empty(shp, dtype=torch.uint8, device=dev), torch.empty(shp, dtype=torch.uint8, device=dev)) for _ in range(slots)]
d_out = [(torch.empty(shp, dtype=torch.float32, device=dev), torch.empty(shp, dtype=torch.float32, device=dev)) for _ in range(slots)]
ws = [hsflow.alloc_workspace(rows, cols, batch, dev) for _ in range(slots)]
for sl in range(slots):
    d_in[sl][0].copy_(hA); d_in[sl][1].copy_(hB)
torch.cuda.synchronize()
def solve(sl, s):
    hsflow.flow_device(d_in[sl][0], d_in[sl][1], 5, iters, 1.0, d_out[sl][0], d_out[sl][1], ws[sl], s)
graphs = []
cur = torch.cuda.current_stream(dev)
for sl in range(slots):
    cap = torch.cuda.Stream(dev); cap.wait_stream(cur)
    with torch.cuda.stream(cap):
        solve(sl, cap)
    cur.wait_stream(cap); torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with hsflow.max_streams_as(2), torch.cuda.graph(g, capture_error_mode="thread_local"):
        solve(sl, torch.cuda.current_stream(dev))
    graphs.append(g)
torch.cuda.synchronize()
s_cmp = torch.cuda.Stream(dev)
def timed(fn, reps=20, warm=0.15):
    t = time.perf_counter()
    while time.perf_counter() - t < warm:
        fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps): fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / reps * 1e3, 4)
out = {}
out["slot0_default_stream"] = timed(lambda: graphs[0].replay())
def on_cmp():
    with torch.cuda.stream(s_cmp):
        graphs[0].replay()
out["slot0_on_side_stream"] = timed(on_cmp)
out["slot1_default_stream"] = timed(lambda: graphs[1].replay())
print("RESULT " + json.dumps(out), flush=True)
