"""Interleaved A/B timing of K2 blocking depths / workloads in ONE process
(guide §5.4 rule 24).  Prints one line per (workload, kb) with the median."""
import argparse, json, os, sys, time
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "cpp-optical-flow_amd")]
import numpy as np
import torch
import hsflow

ap = argparse.ArgumentParser()
ap.add_argument("--kbs", default="1,2,4")
ap.add_argument("--workloads", default="1080p:8,4k:2")
ap.add_argument("--window", type=int, default=5)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=40)
ap.add_argument("--dtype", default="f32")
args = ap.parse_args()
sizes = {"1080p": (1080, 1920), "4k": (2160, 3840), "8k": (4320, 7680), "720p": (720, 1280)}
res = {}
setups = []
for wl in args.workloads.split(","):
    name, b = wl.split(":")
    rows, cols = sizes[name]
    b = int(b)
    dt = np.float32 if args.dtype == "f32" else np.uint8
    pairs = [hsflow.synth_pair(1000 + i, rows, cols, dtype=dt) for i in range(b)]
    I0 = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    I1 = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    u = torch.empty(I0.shape, dtype=torch.float32, device="cuda"); v = torch.empty_like(u)
    ws = hsflow.alloc_workspace(rows, cols, b)
    hsflow.gradients_device(I0, I1, ws)
    setups.append((name, b, rows, cols, I0, I1, u, v, ws))
kbs = [int(k) for k in args.kbs.split(",")]
for rnd in range(args.rounds):
    for (name, b, rows, cols, I0, I1, u, v, ws) in setups:
        for kb in kbs:
            hsflow.set_iters_per_launch(kb)
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            hsflow.jacobi_device(rows, cols, b, args.window, args.iters, 1.0, u, v, ws)
            e0.record()
            hsflow.jacobi_device(rows, cols, b, args.window, args.iters, 1.0, u, v, ws)
            e1.record(); torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            res.setdefault((name, b, kb), []).append(ms)
hsflow.set_iters_per_launch(0)
for (name, bb, kb), ts in res.items():
    b = [s for s in setups if s[0] == name and s[1] == bb][0]
    px = b[1] * b[2] * b[3]
    med = float(np.median(ts))
    print(json.dumps({"workload": name, "batch": b[1], "kb": kb, "window": args.window,
                      "ms_median": round(med, 4), "ms_min": round(min(ts), 4),
                      "Mpix_iter_per_s": round(px * args.iters / (med * 1e-3) / 1e6, 1)}))
