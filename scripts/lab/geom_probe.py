"""Single-pair solve times with a lab build of libhsflow (A/B of a launch
geometry): python scripts/lab/geom_probe.py LIB_TAG OUT_DIR.  Writes the
timings and u planes (for a bitwise cross-check) to OUT_DIR."""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import numpy as np
import hsflow
hsflow.LIB_PATH = os.path.join(ROOT, "cpp-optical-flow_amd", "lab", f"libhsflow_{sys.argv[1]}.so")
import torch

SHAPES = [("1080p_w5", 1080, 1920, 5, 300, 1), ("1080p_w3", 1080, 1920, 3, 300, 1),
          ("720p_x2", 720, 1280, 5, 300, 2), ("kitti", 375, 1242, 5, 100, 1),
          ("4k", 2160, 3840, 5, 500, 1), ("1080p_x8", 1080, 1920, 5, 300, 8),
          ("4k_x2", 2160, 3840, 5, 500, 2)]
ALL = list(SHAPES)
if len(sys.argv) > 3 and sys.argv[3]:  # a subset: comma-separated tags
    SHAPES = [s for s in SHAPES if s[0] in sys.argv[3].split(",")]


def timed(I0, I1, w, iters, reps=20):
    rows, cols = I0.shape[-2:]
    b = I0.shape[0]
    ws = hsflow.alloc_workspace(rows, cols, b)
    u = torch.empty(b, rows, cols, device="cuda")
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
    return e0.elapsed_time(e1) / reps, u


out = {}
os.makedirs(sys.argv[2], exist_ok=True)
if len(sys.argv) > 4:  # an explicit order, repeats allowed
    SHAPES = [next(s for s in ALL if s[0] == t) for t in sys.argv[4].split(",")]
for tag, rows, cols, w, iters, b in SHAPES:
    ps = [hsflow.synth_pair(1000 + i, rows, cols) for i in range(b)]
    I0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
    I1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
    ms, u = timed(I0, I1, w, iters)
    np.save(os.path.join(sys.argv[2], f"{sys.argv[1]}_{tag}.npy"), u.cpu().numpy())
    out[tag] = {"ms": round(ms, 4), "Mpix_iter_s": round(b * rows * cols * iters / ms / 1e3, 1)}
    print(sys.argv[1], tag, out[tag], flush=True)
with open(os.path.join(sys.argv[2], f"{sys.argv[1]}.json"), "w") as f:
    json.dump(out, f)
