"""Sweep K4 segment heights (hsflow_set_strip_rows) on the bench workloads:
graph-replayed full solves, ms and Mpix*iter/s per setting (0 = automatic),
K2 alongside.  python scripts/k4_sweep.py [--rows-list 0,48,84]"""
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


def timed(I0, I1, window, iters, reps=8):
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
        hsflow.flow_device(I0, I1, window, iters, 1.0, u, v, ws, torch.cuda.current_stream())
    # the bench's pre-warm: the clocks need ~0.1 s of load to settle
    t = time.perf_counter()
    n = 0
    while time.perf_counter() - t < 0.15 and n < 400:
        g.replay()
        n += 1
        if n % 4 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps, u


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows-list", default="0,36,48,60,72,84,96,120")
    ap.add_argument("--cases", default="1080p8,4k2,1080p1,4k1")
    ap.add_argument("--windows", default="5,3")
    ap.add_argument("--streams", type=int, default=0)
    ap.add_argument("--tag", default="")
    ap.add_argument("--kb", type=int, default=0, help="iterations per pass (0 auto)")
    ap.add_argument("--force4", action="store_true", help="K4 even where it does not fill the chip")
    ap.add_argument("--kernel", type=int, default=0,
                    help="pass kernel of the k4 columns (4 = K4, 5 = K5; 0 = automatic)")
    a = ap.parse_args()
    cases = {"1080p8": (8, 1080, 1920, 300), "4k2": (2, 2160, 3840, 500),
             "1080p1": (1, 1080, 1920, 300), "4k1": (1, 2160, 3840, 500),
             "720p1": (1, 720, 1280, 300), "kitti1": (1, 375, 1242, 100),
             "1080p2": (2, 1080, 1920, 300), "8k1": (1, 4320, 7680, 60),
             "1080p32": (32, 1080, 1920, 60), "1080p64": (64, 1080, 1920, 120),
             "1080p32l": (32, 1080, 1920, 120), "1080p16": (16, 1080, 1920, 120),
             "4k8": (8, 2160, 3840, 120), "4k4": (4, 2160, 3840, 120),
             "1080p6": (6, 1080, 1920, 300), "1080p7": (7, 1080, 1920, 300),
             "1080p8f": (8, 1080, 1920, 300), "1080p10": (10, 1080, 1920, 300),
             "1080p12": (12, 1080, 1920, 300), "1080p16f": (16, 1080, 1920, 300),
             # config 5's level-0 row bands at N = 8 / 4 / 2 (extended band,
             # one 24-iteration chunk)
             "band8": (1, 640, 7680, 24), "band4": (1, 1176, 7680, 24),
             "band2": (1, 2208, 7680, 24)}
    hsflow.set_max_streams(a.streams)
    hsflow.set_iters_per_launch(a.kb)
    for name in a.cases.split(","):
        batch, rows, cols, iters = cases[name]
        ps = [hsflow.synth_pair(1000 + i, rows, cols) for i in range(batch)]
        I0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
        I1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
        mp = batch * rows * cols * iters / 1e6
        for w in [int(x) for x in a.windows.split(",")]:
            hsflow.set_jacobi_kernel(2)
            t2, u2 = timed(I0, I1, w, iters)
            hsflow.set_jacobi_kernel(a.kernel or (4 if a.force4 else 0))
            rec = {"tag": a.tag, "kernel": a.kernel, "kb": a.kb, "streams": a.streams, "case": name, "w": w, "k2_ms": round(t2 * 1e3, 3), "k2": round(mp / t2)}
            for n in [int(x) for x in a.rows_list.split(",")]:
                hsflow.set_strip_rows(n)
                t4, u4 = timed(I0, I1, w, iters)
                rec[f"k4_n{n}"] = round(mp / t4)
                if not torch.equal(u2, u4):
                    rec[f"k4_n{n}_MISMATCH"] = True
            hsflow.set_strip_rows(0)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
