"""Which Jacobi kernel and K4 segment height are fastest for launches that
fill part of the chip (single pairs, small batches, config 5's row bands)?
Graph-replayed jacobi_device passes only (gradients once, outside the
timing), 48 iterations (8 passes), after a 0.15 s pre-warm; K2 against K4
at several segment heights, per shape.  Prints one JSON line per shape.
    python scripts/kernel_choice_sweep.py [--rows-list 36,48,60,72,84]
        [--kb-list 4,5 --iters 120]   # also K4 at other depths"""
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

SHAPES = [  # (name, batch, rows, cols)
    ("band8_8k", 1, 640, 7680), ("band4_8k", 1, 1176, 7680), ("band2_8k", 1, 2208, 7680),
    ("band8_4k", 1, 464, 3840), ("band4_4k", 1, 732, 3840), ("band2_4k", 1, 1176, 3840),
    ("4k1", 1, 2160, 3840), ("1080p1", 1, 1080, 1920), ("1080p2", 2, 1080, 1920),
    ("1080p4", 4, 1080, 1920), ("720p4", 4, 720, 1280), ("kitti2", 2, 375, 1242),
    ("1080p3", 3, 1080, 1920), ("1080p5", 5, 1080, 1920), ("1080p6", 6, 1080, 1920),
    ("1080p7", 7, 1080, 1920), ("1080p8", 8, 1080, 1920), ("4k2", 2, 2160, 3840),
    # shapes no rule was fitted on (a check for regressions)
    ("720p8", 8, 720, 1280), ("720p2", 2, 720, 1280), ("1440p2", 2, 1440, 2560),
    ("1440p1", 1, 1440, 2560), ("4k3", 3, 2160, 3840), ("1080p12", 12, 1080, 1920),
    ("kitti8", 8, 375, 1242), ("5k1", 1, 2880, 5120),
    # config 5's extended 2-D blocks (blocks.plan2d, chunks 48/96): N = 8
    # (2 x 4) and N = 4 (2 x 2) interior blocks of levels 0 and 1, N = 2
    ("blk8_l0", 1, 2256, 2112), ("blk8_l1", 1, 1272, 1344), ("blk4_l0", 1, 2256, 3936),
    ("blk4_l1", 1, 1272, 2112), ("blk2_l0", 1, 4320, 3936), ("blk2_l1", 1, 2160, 2112),
    # config 5's 8K level 0 on one GPU (two rounds of waves at 84 rows)
    ("8k1", 1, 4320, 7680),
]


def timed_passes(rows, cols, batch, iters, kernel, seg_rows, ws, u, v, kb=0):
    hsflow.set_jacobi_kernel(kernel)
    hsflow.set_strip_rows(seg_rows)
    hsflow.set_iters_per_launch(kb)
    try:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            hsflow.jacobi_device(rows, cols, batch, 5, iters, 1.0, u, v, ws, warm_start=True, stream=s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with hsflow.max_streams_as(2), torch.cuda.graph(g, capture_error_mode="thread_local"):
            hsflow.jacobi_device(rows, cols, batch, 5, iters, 1.0, u, v, ws, warm_start=True,
                                 stream=torch.cuda.current_stream())
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
        for _ in range(20):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 20
    finally:
        hsflow.set_jacobi_kernel(0)
        hsflow.set_strip_rows(0)
        hsflow.set_iters_per_launch(0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows-list", default="36,48,60,72,84")
    ap.add_argument("--iters", type=int, default=48)
    ap.add_argument("--shapes", default="")
    # K4 depths to sweep besides the default (round 6: w = 5 K4 is built at
    # KB 4, 5 and 6; use --iters divisible by each, e.g. 120)
    ap.add_argument("--kb-list", default="")
    a = ap.parse_args()
    want = set(a.shapes.split(",")) if a.shapes else None
    for name, batch, rows, cols in SHAPES:
        if want and name not in want:
            continue
        ps = [hsflow.synth_pair(1000 + i, rows, cols) for i in range(batch)]
        I0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
        I1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
        ws = hsflow.alloc_workspace(rows, cols, batch)
        hsflow.gradients_device(I0, I1, ws)
        u = torch.zeros((batch, rows, cols), dtype=torch.float32, device="cuda")
        v = torch.zeros_like(u)
        mp = batch * rows * cols * a.iters / 1e6
        rec = {"shape": name, "batch": batch, "rows": rows, "cols": cols,
               "auto": hsflow.jacobi_kernel_name(rows, cols, batch, 5)}
        t0 = timed_passes(rows, cols, batch, a.iters, 0, 0, ws, u, v)
        rec["auto_ms"] = round(t0, 4)
        rec["k2_ms"] = round(timed_passes(rows, cols, batch, a.iters, 2, 0, ws, u, v), 4)
        for n in [int(x) for x in a.rows_list.split(",")]:
            rec[f"k4_{n}_ms"] = round(timed_passes(rows, cols, batch, a.iters, 4, n, ws, u, v), 4)
        for kb in [int(x) for x in a.kb_list.split(",") if x]:
            for n in [int(x) for x in a.rows_list.split(",")]:
                rec[f"k4kb{kb}_{n}_ms"] = round(
                    timed_passes(rows, cols, batch, a.iters, 4, n, ws, u, v, kb=kb), 4)
        best = min((k for k in rec if k.endswith("_ms")), key=lambda k: rec[k])
        rec["best"] = best
        rec["auto_over_best"] = round(rec["auto_ms"] / rec[best], 3)
        rec["Mpix_iter_s_best"] = round(mp / rec[best] * 1e3)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
