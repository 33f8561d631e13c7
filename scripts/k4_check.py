"""K4 (streaming strips) against K2 (register tiles) on the GPU: bit-identical
(u, v) on a spread of shapes, windows, lengths, warm starts and gradient
formats, then graph-replayed solve times of both on the bench workloads.

    python scripts/k4_check.py [--quick]

Development check (the parity suite proper is tests/test_gpu_parity.py and
tests/test_strips.py)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import hsflow  # noqa: E402


def solve(kernel, I0, I1, window, iters, warm=None):
    hsflow.set_jacobi_kernel(kernel)
    try:
        if warm is None:
            u, v = hsflow.flow_device(I0, I1, window, iters, 1.0)
        else:
            rows, cols = I0.shape[-2:]
            batch = I0.shape[0]
            ws = hsflow.alloc_workspace(rows, cols, batch, I0.device)
            hsflow.gradients_device(I0, I1, ws)
            u, v = warm[0].clone(), warm[1].clone()
            hsflow.jacobi_device(rows, cols, batch, window, iters, 1.0, u, v, ws,
                                 warm_start=True)
        torch.cuda.synchronize()
        return u, v
    finally:
        hsflow.set_jacobi_kernel(0)


def pairs(batch, rows, cols, nonint=()):
    ps = [hsflow.synth_pair(1000 + i, rows, cols) for i in range(batch)]
    I0 = np.stack([p[0] for p in ps])
    I1 = np.stack([p[1] for p in ps])
    for i in nonint:  # non-integral frames: the f32-gradient path
        I0[i] += 0.25
    return torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()


def timed(kernel, I0, I1, window, iters, reps=5):
    hsflow.set_jacobi_kernel(kernel)
    rows, cols = I0.shape[-2:]
    u = torch.empty(I0.shape, dtype=torch.float32, device="cuda")
    v = torch.empty_like(u)
    ws = hsflow.alloc_workspace(rows, cols, I0.shape[0], "cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        hsflow.flow_device(I0, I1, window, iters, 1.0, u, v, ws, s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with hsflow.max_streams_as(2), torch.cuda.graph(g):
        hsflow.flow_device(I0, I1, window, iters, 1.0, u, v, ws,
                           torch.cuda.current_stream())
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    hsflow.set_jacobi_kernel(0)
    return dt, u


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    args = ap.parse_args()
    cases = [
        (1, 1, 1, 5, 12), (1, 2, 3, 5, 7), (2, 37, 53, 5, 13), (1, 300, 49, 3, 17),
        (3, 64, 130, 5, 12), (2, 101, 333, 3, 24), (1, 375, 1242, 5, 100),
        (1, 375, 1242, 3, 100), (2, 200, 257, 5, 30), (1, 90, 256, 5, 6),
        (8, 1080, 1920, 5, 24), (2, 2160, 3840, 5, 18), (8, 1080, 1920, 3, 16),
    ]
    bad = 0
    for batch, rows, cols, w, iters in cases:
        I0, I1 = pairs(batch, rows, cols)
        a = solve(2, I0, I1, w, iters)
        b = solve(4, I0, I1, w, iters)
        same = torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
        diff = float((a[0] - b[0]).abs().max())
        print(f"{batch}x{rows}x{cols} w{w} it{iters} kernel={hsflow.jacobi_kernel_name(rows, cols, batch, w)}"
              f" identical={same} maxdiff={diff:.3g}", flush=True)
        bad += not same
    # warm start, mixed f32-gradient batch
    I0, I1 = pairs(3, 120, 200, nonint=(1,))
    w0 = (torch.randn(3, 120, 200, device="cuda"), torch.randn(3, 120, 200, device="cuda"))
    for w in (3, 5):
        a = solve(2, I0, I1, w, 24, warm=w0)
        b = solve(4, I0, I1, w, 24, warm=w0)
        same = torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
        print(f"warm+f32 mixed w{w} identical={same}", flush=True)
        bad += not same
    out = {"mismatches": bad}
    if not args.quick:
        for name, (batch, rows, cols, iters) in {"1080p x8": (8, 1080, 1920, 300),
                                                  "4k x2": (2, 2160, 3840, 500),
                                                  "1080p x1": (1, 1080, 1920, 300),
                                                  "4k x1": (1, 2160, 3840, 500)}.items():
            I0, I1 = pairs(batch, rows, cols)
            for w in (5, 3):
                t2, u2 = timed(2, I0, I1, w, iters)
                t4, u4 = timed(4, I0, I1, w, iters)
                mp = batch * rows * cols * iters / 1e6
                rec = {"case": name, "w": w, "k2_ms": round(t2 * 1e3, 3),
                       "k4_ms": round(t4 * 1e3, 3), "k2_Mpix_it_s": round(mp / t2),
                       "k4_Mpix_it_s": round(mp / t4), "identical": bool(torch.equal(u2, u4))}
                print(json.dumps(rec), flush=True)
                bad += not rec["identical"]
    print(json.dumps({"mismatches": bad}))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
