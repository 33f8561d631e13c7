"""K4 rectangle vs parallelogram segments (hsflow_set_strip_segments 1 / 2),
same process, alternated: bit equality of (u, v) and graph-replayed solve
times on the bench workloads.

    python scripts/lab/pg_ab.py [--rounds 3]          # GPU box
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import hsflow  # noqa: E402

SHAPES = (("1080p8", 8, 1080, 1920, 300, 5), ("4k2", 2, 2160, 3840, 500, 5),
          ("4k1", 1, 2160, 3840, 500, 5), ("1080p8w3", 8, 1080, 1920, 300, 3),
          ("1080p1", 1, 1080, 1920, 300, 5))


SEG_ROWS = 0
KERNEL = 0


def graph_for(mode, I0, I1, window, iters, u, v, ws):
    hsflow.set_strip_segments(mode)
    hsflow.set_strip_rows(SEG_ROWS)
    hsflow.set_jacobi_kernel(KERNEL)
    try:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            hsflow.flow_device(I0, I1, window, iters, 1.0, u, v, ws, s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with hsflow.max_streams_as(2), torch.cuda.graph(g, capture_error_mode="thread_local"):
            hsflow.flow_device(I0, I1, window, iters, 1.0, u, v, ws,
                               torch.cuda.current_stream())
        return g
    finally:
        hsflow.set_strip_segments(0)
        hsflow.set_strip_rows(0)
        hsflow.set_jacobi_kernel(0)


def timed(g, steps=20):
    t = time.perf_counter()
    n = 0
    while time.perf_counter() - t < 0.15:
        g.replay()
        n += 1
        if n % 4 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default="")
    ap.add_argument("--only", type=int, default=0,
                    help="time one mode only (1 rectangles, 2 parallelograms), for A/Bs "
                         "in separate processes")
    ap.add_argument("--seg", type=int, default=0, help="K4 segment rows (0: automatic)")
    ap.add_argument("--kernel", type=int, default=0, help="hsflow_set_jacobi_kernel")
    args = ap.parse_args()
    global SEG_ROWS, KERNEL
    SEG_ROWS, KERNEL = args.seg, args.kernel
    out = {}
    for tag, batch, rows, cols, iters, window in SHAPES:
        if args.shapes and tag not in args.shapes.split(","):
            continue
        ps = [hsflow.synth_pair(1000 + i, rows, cols) for i in range(batch)]
        I0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
        I1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
        res = {}
        outs = {}
        graphs = {}
        modes = (args.only,) if args.only else (1, 2)
        for mode in modes:
            u = torch.empty((batch, rows, cols), dtype=torch.float32, device="cuda")
            v = torch.empty_like(u)
            ws = hsflow.alloc_workspace(rows, cols, batch)
            # ws stays referenced: the graph replays into it
            graphs[mode] = (graph_for(mode, I0, I1, window, iters, u, v, ws), u, v, ws)
            res[mode] = []
        for r in range(args.rounds):
            for mode in (modes if r % 2 == 0 else modes[::-1]):
                g, u, v, _ = graphs[mode]
                u.fill_(float("nan"))
                v.fill_(float("nan"))
                res[mode].append(timed(g))
                outs[mode] = (u.clone(), v.clone())
        mpx = batch * rows * cols * iters / 1e3
        if args.only:
            out[tag] = {"mode": args.only, "ms": [round(x, 4) for x in res[args.only]],
                        "M": round(mpx / min(res[args.only]) / 1e6, 4),
                        "u_sum": float(outs[args.only][0].double().sum())}
            print(tag, json.dumps(out[tag]), flush=True)
            continue
        same = bool(torch.equal(outs[1][0], outs[2][0]) and torch.equal(outs[1][1], outs[2][1]))
        nd = int((outs[1][0] != outs[2][0]).sum() + (outs[1][1] != outs[2][1]).sum())
        out[tag] = {"rect_ms": [round(x, 4) for x in res[1]],
                    "pg_ms": [round(x, 4) for x in res[2]],
                    "rect_M": round(mpx / min(res[1]) / 1e6, 4),
                    "pg_M": round(mpx / min(res[2]) / 1e6, 4),
                    "gain": round(min(res[1]) / min(res[2]) - 1, 4),
                    "bit_identical": same, "differing": nd,
                    "finite": bool(torch.isfinite(outs[2][0]).all())}
        print(tag, json.dumps(out[tag]), flush=True)
    print("RESULT " + json.dumps(out), flush=True)
    return 0 if all(v.get("bit_identical", True) for v in out.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
