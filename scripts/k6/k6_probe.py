"""K6 (resident solve) vs K2 (one launch per pass) on single pairs: same-box
A/B of the whole solve (hipGraph replay, inputs resident), bit-identity
checked.  Usage: python scripts/k6_probe.py [out.json]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cpp-optical-flow_amd"))
import numpy as np
import torch
import hsflow

SHAPES = [("1080p", 1080, 1920, 5, 300, 1), ("1080p_w3", 1080, 1920, 3, 300, 1),
          ("720p", 720, 1280, 5, 300, 1), ("kitti", 375, 1242, 5, 100, 1),
          ("1080p_kb6", 1080, 1920, 5, 300, 6)]


def timed(kernel, kb, I0, I1, w, iters, reps=30):
    hsflow.set_jacobi_kernel(kernel)
    hsflow.set_iters_per_launch(0 if kb == 1 else kb)
    rows, cols = I0.shape[-2:]
    try:
        name = hsflow.jacobi_kernel_name(rows, cols, 1, w)
        ws = hsflow.alloc_workspace(rows, cols, 1)
        u = torch.empty(1, rows, cols, device="cuda")
        v = torch.empty_like(u)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            hsflow.flow_device(I0, I1, w, iters, 1.0, u, v, ws, s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            hsflow.flow_device(I0, I1, w, iters, 1.0, u, v, ws, s)
        t_end = time.perf_counter() + 0.3
        while time.perf_counter() < t_end:
            g.replay()
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        u.fill_(float("nan"))
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        return name, ms, u.clone(), v.clone()
    finally:
        hsflow.set_jacobi_kernel(0)
        hsflow.set_iters_per_launch(0)


def main():
    out = {}
    for tag, rows, cols, w, iters, kb in SHAPES:
        a, b = hsflow.synth_pair(1000, rows, cols)
        I0 = torch.from_numpy(a)[None].cuda()
        I1 = torch.from_numpy(b)[None].cuda()
        n2, ms2, u2, v2 = timed(2, kb, I0, I1, w, iters)
        n6, ms6, u6, v6 = timed(6, kb, I0, I1, w, iters)
        same = bool(torch.equal(u2, u6) and torch.equal(v2, v6))
        mp = rows * cols * iters / 1e6
        out[tag] = {"k2": n2, "k2_ms": round(ms2, 4), "k2_Mpix_iter_s": round(mp / ms2 * 1e3, 1),
                    "k6": n6, "k6_ms": round(ms6, 4), "k6_Mpix_iter_s": round(mp / ms6 * 1e3, 1),
                    "bit_identical": same}
        print(tag, json.dumps(out[tag]), flush=True)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
