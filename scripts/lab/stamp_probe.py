"""Per-workgroup timeline of one K2 pass of a single 1080p pair (lab build
with s_memrealtime stamps, 100 MHz): kernel start, slab loaded + operator
set up, first iteration done, last iteration's stores issued, stores drained.
python scripts/lab/stamp_probe.py [w] [lab tag]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import numpy as np
import hsflow
hsflow.LIB_PATH = os.path.join(ROOT, "cpp-optical-flow_amd", "lab",
                               f"libhsflow_{sys.argv[2] if len(sys.argv) > 2 else 'stamp'}.so")
import torch

w = int(sys.argv[1]) if len(sys.argv) > 1 else 5
rows, cols = 1080, 1920
a, b = hsflow.synth_pair(1000, rows, cols)
I0, I1 = torch.from_numpy(a)[None].cuda(), torch.from_numpy(b)[None].cuda()
ws = hsflow.alloc_workspace(rows, cols, 1)
u = torch.empty(1, rows, cols, device="cuda")
v = torch.empty_like(u)
hsflow.gradients_device(I0, I1, ws)
t_end = time.perf_counter() + 0.5
while time.perf_counter() < t_end:
    hsflow.jacobi_device(rows, cols, 1, w, 300, 1.0, u, v, ws)
    torch.cuda.synchronize()
res = {}
for iters in (8, 16):
    hsflow.jacobi_device(rows, cols, 1, w, iters, 1.0, u, v, ws)
    torch.cuda.synchronize()
    buf = np.zeros((4096, 8), dtype=np.uint64)
    assert hsflow.lib().hsflow_lab_stamps(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    st = buf[np.any(buf != 0, axis=1)].astype(np.int64)
    st = st[st[:, 0] > 0]
    t0 = st[:, 0].min()
    rel = (st[:, :5] - t0) / 100.0  # us
    q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 50, 100)]
    res[iters] = {"workgroups": int(len(st)), "start_us": q(rel[:, 0]),
                  "loaded_setup_us": q(rel[:, 1] - rel[:, 0]),
                  "first_iter_us": q(rel[:, 2] - rel[:, 1]),
                  "rest_iters_us": q(rel[:, 3] - rel[:, 2]),
                  "drain_us": q(rel[:, 4] - rel[:, 3]),
                  "end_us": q(rel[:, 4])}
    print(iters, json.dumps(res[iters]), flush=True)
    if iters == 16:  # per tile: where are the slow ones?
        info = buf[np.any(buf != 0, axis=1)][:, 5].astype(np.int64)
        info = info[st[:, 0] > 0] if len(info) == len(st) else info
        tx, ty = info & 0xFFFF, (info >> 16) & 0xFFFF
        edge, rowe = (info >> 32) & 1, (info >> 33) & 1
        end = rel[:, 4]
        it = rel[:, 3] - rel[:, 2]
        for name, m in (("interior", edge == 0), ("edge_cols", (edge == 1) & (rowe == 0)),
                        ("edge_rows", (edge == 1) & (rowe == 1))):
            if m.any():
                print(" ", name, int(m.sum()), "rest_iters", q(it[m]), "end", q(end[m]), flush=True)
        slow = np.argsort(-end)[:8]
        print("  slowest", [(int(tx[i]), int(ty[i]), round(float(end[i]), 2)) for i in slow], flush=True)
