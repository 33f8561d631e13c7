"""Config 5 in row bands with K virtual ranks on ONE GPU (LocalComm: the
exchange is an in-process copy), plain vs overlapped schedule: what the
overlap costs in extra rows and what concurrency it gets on one device.
(The exchange it hides only exists with N GPUs.)  Checks both against the
single-GPU pyramid solve bit for bit.
    python scripts/bands_overlap_probe.py [--ranks 8] [--chunk 12] [--iters 1000]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import torch  # noqa: E402
import hsflow  # noqa: E402
import row_bands as rb  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ranks", type=int, default=8)
ap.add_argument("--chunk", type=int, default=12)
ap.add_argument("--iters", type=int, default=1000)
a = ap.parse_args()
I0, I1 = hsflow.synth_pair(1000, 4320, 7680)
t0 = torch.from_numpy(I0).cuda().half()
t1 = torch.from_numpy(I1).cuda().half()
ref = hsflow.flow_pyramid_device(t0, t1, 3, 5, a.iters, 1.0)
torch.cuda.synchronize()
p = rb.plan(4320, 7680, 3, a.ranks, 5, a.chunk)
out = {"ranks": a.ranks, "chunk": a.chunk, "halo": p.halo, "iters_per_level": a.iters}
for name, solve in (("plain", rb.solve), ("overlapped", rb.solve_overlapped)):
    ops = [rb.DeviceOps(5, 1.0, t0.device) for _ in range(a.ranks)]
    comm = rb.LocalComm()
    for rep in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        st = solve([t0] * a.ranks, [t1] * a.ranks, p, a.iters, ops, comm, list(range(a.ranks)))
        u, v = rb.gather_owned(st, p, comm)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
    out[name] = {"ms": round(dt * 1e3, 2), "bit_identical": bool(torch.equal(u, ref[0]) and
                                                                 torch.equal(v, ref[1]))}
    print(name, out[name], flush=True)
print(json.dumps(out))
