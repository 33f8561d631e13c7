"""Same-box A/B timing of one library build (HSFLOW_LIB selects it; probe
builds honour HSFLOW_* switches): a bench-shaped solve (K1 + every K2 pass)
captured into a hipGraph and replayed.  Prints one JSON line per workload.

    HSFLOW_LIB=... python scripts/solve_ab.py --tag NAME [--window 5] [--reps 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import hsflow  # noqa: E402

WL = {"1080p": (1080, 1920, 300, 8), "4k": (2160, 3840, 500, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="")
    ap.add_argument("--window", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--workloads", default="1080p,4k")
    a = ap.parse_args()
    for name in a.workloads.split(","):
        rows, cols, iters, batch = WL[name]
        ps = [hsflow.synth_pair(1000 + i, rows, cols) for i in range(batch)]
        I0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
        I1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
        u, v = torch.empty_like(I0), torch.empty_like(I0)
        ws = hsflow.alloc_workspace(rows, cols, batch)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            hsflow.flow_device(I0, I1, a.window, iters, 1.0, u, v, ws, s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            hsflow.flow_device(I0, I1, a.window, iters, 1.0, u, v, ws,
                               torch.cuda.current_stream())
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.reps):
            g.replay()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.reps
        print(json.dumps({"tag": a.tag, "workload": name, "window": a.window,
                          "Mpix_iter_per_s": round(batch * rows * cols * iters / dt / 1e6, 1),
                          "ms_per_solve": round(dt * 1e3, 3),
                          "u_sum": float(u.double().sum())}), flush=True)
        del I0, I1, u, v, ws, g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
