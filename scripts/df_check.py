"""Dataflow K2 (hsflow_set_jacobi_kernel(4)) against per-pass K2 launches
(kernel 2): bit-identical (u, v) on batches 1-16, ragged shapes, warm
starts, and hipGraph capture; reports the dependency-timeout word.
    HSFLOW_LIB=... python scripts/df_check.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import hsflow  # noqa: E402


def solve(kernel, I0, I1, iters, warm=None):
    hsflow.set_jacobi_kernel(kernel)
    try:
        if warm is None:
            u, v = hsflow.flow_device(I0, I1, 5, iters, 1.0)
        else:
            rows, cols = I0.shape[-2:]
            batch = I0.shape[0]
            ws = hsflow.alloc_workspace(rows, cols, batch)
            hsflow.gradients_device(I0, I1, ws)
            u, v = warm[0].clone(), warm[1].clone()
            hsflow.jacobi_device(rows, cols, batch, 5, iters, 1.0, u, v, ws, warm_start=True)
        torch.cuda.synchronize()
        return u, v
    finally:
        hsflow.set_jacobi_kernel(0)


bad = 0
cases = [(1, 96, 160, 30), (3, 120, 210, 37), (8, 1080, 1920, 300), (16, 200, 330, 13),
         (2, 2160, 3840, 12), (9, 64, 64, 7), (8, 61, 77, 25), (1, 1, 1, 6)]
for batch, rows, cols, iters in cases:
    ps = [hsflow.synth_pair(3000 + k, rows, cols) for k in range(batch)]
    I0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
    I1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
    a = solve(2, I0, I1, iters)
    b = solve(4, I0, I1, iters)
    ok = torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    print(f"batch {batch} {rows}x{cols} it {iters}: {'bit-identical' if ok else 'MISMATCH'}",
          flush=True)
    bad += not ok
    if batch <= 3 and rows < 300:  # warm start and f32 (non-integral) inputs
        w = (torch.rand_like(a[0]), torch.rand_like(a[1]))
        a2 = solve(2, I0, I1, iters, warm=w)
        b2 = solve(4, I0, I1, iters, warm=w)
        ok2 = torch.equal(a2[0], b2[0]) and torch.equal(a2[1], b2[1])
        J0, J1 = I0 + 0.25, I1 * 0.5
        a3 = solve(2, J0, J1, iters)
        b3 = solve(4, J0, J1, iters)
        ok3 = torch.equal(a3[0], b3[0]) and torch.equal(a3[1], b3[1])
        print(f"   warm start {'ok' if ok2 else 'MISMATCH'}, f32 gradients {'ok' if ok3 else 'MISMATCH'}",
              flush=True)
        bad += (not ok2) + (not ok3)
# graph capture of the dataflow solve (memset + one launch), replayed
ps = [hsflow.synth_pair(4000 + k, 1080, 1920) for k in range(8)]
I0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
I1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
ref = solve(2, I0, I1, 300)
hsflow.set_jacobi_kernel(4)
u, v = torch.empty_like(I0), torch.empty_like(I0)
ws = hsflow.alloc_workspace(1080, 1920, 8)
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    hsflow.flow_device(I0, I1, 5, 300, 1.0, u, v, ws, s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, capture_error_mode="thread_local"):
    hsflow.flow_device(I0, I1, 5, 300, 1.0, u, v, ws, torch.cuda.current_stream())
for _ in range(3):
    u.zero_()
    g.replay()
torch.cuda.synchronize()
hsflow.set_jacobi_kernel(0)
okg = torch.equal(u, ref[0]) and torch.equal(v, ref[1])
print(f"graph replay x3: {'bit-identical' if okg else 'MISMATCH'}", flush=True)
bad += not okg
print("DF CHECK", "PASS" if bad == 0 else f"FAIL ({bad})")
sys.exit(1 if bad else 0)
