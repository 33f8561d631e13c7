"""Config 5 in row bands with K virtual ranks on ONE GPU (LocalComm: the
exchange is an in-process copy), plain vs overlapped schedule, each run
eagerly (one host call per operation) and as one captured hipGraph
(row_bands.graphed: no host time), with all virtual ranks on the caller's
stream or (eagerly) each on a stream of its own.  Every variant is checked against the
single-GPU pyramid solve bit for bit.  (The exchange the overlap hides only
exists with N GPUs; on one device the overlapped schedule pays 3 halos of
extra rows per band edge and gains concurrency.)
    python scripts/bands_overlap_probe.py [--ranks 8] [--chunk 12] [--iters 1000]"""
import argparse
import faulthandler
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import torch  # noqa: E402
import hsflow  # noqa: E402
import row_bands as rb  # noqa: E402

faulthandler.enable()
ap = argparse.ArgumentParser()
ap.add_argument("--ranks", type=int, default=8)
ap.add_argument("--chunk", type=int, default=12)
ap.add_argument("--iters", type=int, default=1000)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--no-eager", action="store_true")
ap.add_argument("--modes", default="plain_shared,overlapped_shared,plain_per_rank,"
                "overlapped_per_rank")
a = ap.parse_args()
I0, I1 = hsflow.synth_pair(1000, 4320, 7680)
t0 = torch.from_numpy(I0).cuda().half()
t1 = torch.from_numpy(I1).cuda().half()
ref = hsflow.flow_pyramid_device(t0, t1, 3, 5, a.iters, 1.0)
torch.cuda.synchronize()
# the undivided solve, graph-replayed, for scale
g1 = torch.cuda.CUDAGraph()
u1, v1 = torch.empty_like(ref[0]), torch.empty_like(ref[1])
pws = torch.empty(hsflow.pyramid_workspace_bytes(4320, 7680, 1, 3), dtype=torch.uint8,
                  device="cuda")
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    hsflow.flow_pyramid_device(t0, t1, 3, 5, a.iters, 1.0, u1, v1, pws, s)
torch.cuda.synchronize()
with torch.cuda.graph(g1):
    hsflow.flow_pyramid_device(t0, t1, 3, 5, a.iters, 1.0, u1, v1, pws,
                               torch.cuda.current_stream())
g1.replay()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(a.reps):
    g1.replay()
torch.cuda.synchronize()
p = rb.plan(4320, 7680, 3, a.ranks, 5, a.chunk)
out = {"ranks": a.ranks, "chunk": a.chunk, "halo": p.halo, "iters_per_level": a.iters,
       "undivided_graph_ms": round((time.perf_counter() - t) / a.reps * 1e3, 2),
       "undivided_bit_identical": bool(torch.equal(u1, ref[0]) and torch.equal(v1, ref[1]))}
print(json.dumps(out), flush=True)
for streams in ("shared", "per_rank"):
    for name, solver in (("plain", rb.solve), ("overlapped", rb.solve_overlapped)):
        if f"{name}_{streams}" not in a.modes.split(","):
            continue
        def mk():
            return [rb.DeviceOps(5, 1.0, t0.device,
                                 stream=torch.cuda.Stream() if streams == "per_rank" else None)
                    for _ in range(a.ranks)]
        rec = {}
        if not a.no_eager:
            ops, comm = mk(), rb.LocalComm()
            for rep in range(2):
                torch.cuda.synchronize()
                t = time.perf_counter()
                st = solver([t0] * a.ranks, [t1] * a.ranks, p, a.iters, ops, comm,
                            list(range(a.ranks)))
                u, v = rb.gather_owned(st, p, comm)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t
            rec["eager_ms"] = round(dt * 1e3, 2)
            rec["eager_bit_identical"] = bool(torch.equal(u, ref[0]) and torch.equal(v, ref[1]))
            del st, u, v
        if streams == "per_rank":  # rb.graphed: caller's stream only
            out[f"{name}_{streams}"] = rec
            print(name, streams, json.dumps(rec), flush=True)
            continue
        ops, comm = mk(), rb.LocalComm()
        t = time.perf_counter()
        g, u, v = rb.graphed(solver, [t0] * a.ranks, [t1] * a.ranks, p, a.iters, ops, comm,
                             list(range(a.ranks)))
        torch.cuda.synchronize()
        rec["capture_s"] = round(time.perf_counter() - t, 2)
        u.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.reps):
            g.replay()
        torch.cuda.synchronize()
        rec["graph_ms"] = round((time.perf_counter() - t) / a.reps * 1e3, 2)
        rec["graph_bit_identical"] = bool(torch.equal(u, ref[0]) and torch.equal(v, ref[1]))
        out[f"{name}_{streams}"] = rec
        print(name, streams, json.dumps(rec), flush=True)
        del g, u, v
        torch.cuda.empty_cache()
print(json.dumps(out))
