"""The bench's timed step on its own, for rocprofv3 kernel traces and --pmc
counter passes of exactly the configuration bench.py times: one full solve
of a resident batch (K1 + the Jacobi passes, the batch split over the
library's side streams), captured once into a hipGraph and replayed `reps`
times, as bench.resident_leg does.

    python scripts/timed_step.py --rows 1080 --cols 1920 --batch 8 --iters 300 --reps 5

Prints one line: kernel, blocking depth, passes per solve and the mean wall
time per replay (events around the replays) -- scripts/pmc_collect.py reads
it next to the profiler output."""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import hsflow  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1080)
    ap.add_argument("--cols", type=int, default=1920)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--window", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--warm-s", type=float, default=0.15,
                    help="untimed replays first (the bench's pre-warm)")
    a = ap.parse_args()
    ps = [hsflow.synth_pair(1000 + i, a.rows, a.cols) for i in range(a.batch)]
    I0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
    I1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
    u = torch.empty((a.batch, a.rows, a.cols), dtype=torch.float32, device="cuda")
    v = torch.empty_like(u)
    ws = hsflow.alloc_workspace(a.rows, a.cols, a.batch)
    cur = torch.cuda.current_stream()
    cap = torch.cuda.Stream()
    cap.wait_stream(cur)
    with torch.cuda.stream(cap):
        hsflow.flow_device(I0, I1, a.window, a.iters, 1.0, u, v, ws, cap)
    cur.wait_stream(cap)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with hsflow.max_streams_as(2), torch.cuda.graph(g, capture_error_mode="thread_local"):
        hsflow.flow_device(I0, I1, a.window, a.iters, 1.0, u, v, ws,
                           torch.cuda.current_stream())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < a.warm_s and n < 400:
        g.replay()
        n += 1
        if n % 4 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    kb = hsflow.iters_per_launch(a.rows, a.cols, a.batch, a.window)
    print("kernel", hsflow.jacobi_kernel_name(a.rows, a.cols, a.batch, a.window),
          "kb", kb, "passes", -(-a.iters // kb), "prewarm", n, "reps", a.reps,
          "ms_per_step", round(e0.elapsed_time(e1) / a.reps, 4),
          "finite", bool(torch.isfinite(u).all()), flush=True)


if __name__ == "__main__":
    main()
