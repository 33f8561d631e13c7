"""Run Jacobi passes of one workload on one stream, for rocprofv3 counter
passes (scripts/gpu_k4_pmc.sh) and kernel traces: K1 once, then `reps`
full solves' worth of single-stream Jacobi launches with the chosen kernel.

    python scripts/k2k4_passes.py --kernel 4 --rows 1080 --cols 1920 --batch 8 \
        --iters 300 --window 5 --reps 2
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import hsflow  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", type=int, default=0)
    ap.add_argument("--rows", type=int, default=1080)
    ap.add_argument("--cols", type=int, default=1920)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--window", type=int, default=5)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--f16", action="store_true")
    ap.add_argument("--segments", type=int, default=0,
                    help="K4 segment shape (needs scripts/k4pg/k4_parallelogram.patch): "
                         "1 rectangles, 2 parallelograms")
    a = ap.parse_args()
    ps = [hsflow.synth_pair(1000 + i, a.rows, a.cols) for i in range(a.batch)]
    I0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
    I1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
    if a.f16:
        I0, I1 = I0.half(), I1.half()
    u = torch.empty((a.batch, a.rows, a.cols), dtype=torch.float32, device="cuda")
    v = torch.empty_like(u)
    ws = hsflow.alloc_workspace(a.rows, a.cols, a.batch)
    hsflow.set_jacobi_kernel(a.kernel)
    hsflow.set_max_streams(1)
    if a.segments:
        hsflow.set_strip_segments(a.segments)
    hsflow.gradients_device(I0, I1, ws)
    for _ in range(a.reps):
        hsflow.jacobi_device(a.rows, a.cols, a.batch, a.window, a.iters, 1.0, u, v, ws)
    torch.cuda.synchronize()
    print("kernel", hsflow.jacobi_kernel_name(a.rows, a.cols, a.batch, a.window),
          "kb", hsflow.iters_per_launch(a.rows, a.cols, a.batch, a.window),
          "finite", bool(torch.isfinite(u).all()), flush=True)


if __name__ == "__main__":
    main()
