"""End-to-end time of the host-buffer API (the getFlow drop-in path) vs the
device solve alone, 1080p u8 pair, f64 (CV_64FC1) and f32 outputs."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cpp-optical-flow_amd"))
import numpy as np
import torch
import hsflow

rows, cols = 1080, 1920
I0, I1 = hsflow.synth_pair(1000, rows, cols, dtype=np.uint8)
ctx = hsflow.Context(0)
for iters in (100, 300):
    for out in (np.float64, np.float32):
        ctx.flow(I0, I1, 5, iters, 1.0, out_dtype=out)
        ts = []
        for _ in range(5):
            t = time.perf_counter()
            ctx.flow(I0, I1, 5, iters, 1.0, out_dtype=out)
            ts.append(time.perf_counter() - t)
        print(f"host API {iters} it, out {np.dtype(out).name}: {1e3 * min(ts):.2f} ms")
    t0, t1 = torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()
    hsflow.set_max_streams(1)
    hsflow.flow_device(t0, t1, 5, iters, 1.0)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        hsflow.flow_device(t0, t1, 5, iters, 1.0)
    torch.cuda.synchronize()
    print(f"device solve {iters} it: {1e3 * (time.perf_counter() - t) / 5:.2f} ms")
    hsflow.set_max_streams(0)
ctx.close()
