"""End-to-end time of the host-buffer API (the getFlow drop-in path) vs the
device solve alone, u8 pairs, f64 (CV_64FC1) and f32 outputs, output
buffers fresh per call or reused (cv::Mat::create keeps them)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cpp-optical-flow_amd"))
import numpy as np
import torch
import hsflow


def med(fn, n=9):
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return 1e3 * sorted(ts)[n // 2]


ctx = hsflow.Context(0)
for rows, cols, iters in ((1080, 1920, 300), (2160, 3840, 500), (1080, 1920, 100)):
    I0, I1 = hsflow.synth_pair(1000, rows, cols, dtype=np.uint8)
    for out in (np.float64, np.float32):
        ctx.flow(I0, I1, 5, iters, 1.0, out_dtype=out)
        fresh = med(lambda: ctx.flow(I0, I1, 5, iters, 1.0, out_dtype=out))
        bufs = (np.empty((rows, cols), out), np.empty((rows, cols), out))
        reuse = med(lambda: ctx.flow(I0, I1, 5, iters, 1.0, out_dtype=out, out=bufs))
        print(f"{cols}x{rows} {iters} it, out {np.dtype(out).name}: fresh {fresh:.3f} ms, "
              f"reused {reuse:.3f} ms", flush=True)
    t0, t1 = torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()
    hsflow.flow_device(t0, t1, 5, iters, 1.0)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        hsflow.flow_device(t0, t1, 5, iters, 1.0)
    torch.cuda.synchronize()
    print(f"{cols}x{rows} device solve {iters} it: {1e3 * (time.perf_counter() - t) / 5:.3f} ms",
          flush=True)
ctx.close()
