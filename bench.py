"""Horn-Schunck throughput bench (BASELINE.json metric: Mpix*iter/s + pairs/s).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload 1080p|4k|8k]

One step = one full solve (K1 gradients + `iters` Jacobi iterations, the
reference's getFlow, hornSchunck.cpp:43-75) of a batch of synthetic frame
pairs per GPU, inputs already resident in HBM (workload 8k = BASELINE config
5: an fp16 7680x4320 pair through the 3-level coarse-to-fine warm start,
`iters` per level; its Mpix*iter counts every level's pixels).  Frame pairs are independent,
so for N > 1 each rank (one process per GPU, torch.distributed over RCCL)
solves its own pairs: weak scaling, no data-path collective (the timing
barrier and max-over-ranks reduction are the only collectives).

Rank 0 prints ONE JSON line.  Besides the driver fields it carries
  roofline      dominant kernel (K2, hs_jacobi_wg_kernel) measured live with
                events on the launch stream; achieved = SURVEY §8(d)'s 28 B
                per pixel-iteration x the pixel-iterations of one launch /
                launch time (> peak is possible: temporal blocking does KB
                iterations per HBM pass); compulsory_* = the 20 B/px one
                blocked pass must move, which PMC `traffic` (committed
                rocprofv3 summary under profiles/, or null) is compared with
                (DESIGN.md "Roofline")
  cpu_baseline  the float64 CPU port (oracle/, mirrors hornSchunck.cpp pass
                by pass) on a bounded sample, 1 thread, rank 0 only
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))

WORKLOADS = {
    # BASELINE.json configs[1] / configs[2]
    "1080p": dict(rows=1080, cols=1920, iters=300, batch=8),
    "4k": dict(rows=2160, cols=3840, iters=500, batch=2),
    # BASELINE.json configs[4] on one GPU (the 8-GPU row-band split is not a
    # bench line; frame-parallel weak scaling is)
    "8k": dict(rows=4320, cols=7680, iters=1000, batch=1, levels=3, dtype="f16"),
}
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="1080p")
    ap.add_argument("--batch", type=int, default=0, help="pairs per GPU per step")
    ap.add_argument("--iters", type=int, default=0)
    ap.add_argument("--window", type=int, default=5)
    ap.add_argument("--alpha", type=float, default=1.0)
    ap.add_argument("--dtype", choices=["f32", "u8", "f16"], default=None,
                    help="input frame element type (default: the workload's, f32 "
                         "for 1080p/4k, f16 for 8k)")
    ap.add_argument("--levels", type=int, default=0,
                    help="pyramid levels (default: the workload's; 1 = plain getFlow)")
    ap.add_argument("--kb", type=int, default=0, help="iterations per K2 launch (0 auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-iters", type=int, default=0,
                    help="Jacobi iterations of the CPU sample (0: auto ~15 s)")
    ap.add_argument("--roofline-reps", type=int, default=3)
    ap.add_argument("--no-graph", action="store_true",
                    help="time eager solves instead of hipGraph replays of one solve")
    ap.add_argument("--mode", choices=["resident", "stream", "bands"], default="resident",
                    help="resident: pairs generated on each rank, already in HBM "
                         "(the metric); stream: BASELINE config 4, rank 0 holds "
                         "--pairs pairs and scatters/gathers them over RCCL; bands: "
                         "BASELINE config 5 on N GPUs, ONE pair split into row bands "
                         "with a halo exchange (row_bands.py)")
    ap.add_argument("--chunk", type=int, default=12,
                    help="bands mode: iterations between halo exchanges")
    ap.add_argument("--pairs", type=int, default=64, help="stream mode: pairs in the stream")
    return ap.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist
    import hsflow

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # HSFLOW_BENCH_BACKEND=gloo + HSFLOW_BENCH_DEVICE=0: rehearse the N > 1
    # logic with several ranks on one GPU (diagnostics; the driver's runs
    # use RCCL, one GPU per rank)
    backend = os.environ.get("HSFLOW_BENCH_BACKEND", "nccl")
    dev = torch.device("cuda", int(os.environ.get("HSFLOW_BENCH_DEVICE", local)))
    torch.cuda.set_device(dev)

    def init_dist():
        if world > 1:
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=dev)
            else:
                dist.init_process_group(backend)

    if args.mode == "stream":
        init_dist()
        return stream_mode(args, world, rank, dev)
    if args.mode == "bands":
        init_dist()
        return bands_mode(args, world, rank, dev)

    wl = dict(WORKLOADS[args.workload])
    rows, cols = wl["rows"], wl["cols"]
    iters = args.iters or wl["iters"]
    batch = args.batch or wl["batch"]
    levels = args.levels or wl.get("levels", 1)
    in_dtype = args.dtype or wl.get("dtype", "f32")
    if args.kb:
        hsflow.set_iters_per_launch(args.kb)

    # synthetic pairs, seed 1000 + global pair index
    np_dtype = np.uint8 if in_dtype == "u8" else np.float32
    pairs = [hsflow.synth_pair(1000 + rank * batch + i, rows, cols, dtype=np_dtype)
             for i in range(batch)]
    I0 = torch.from_numpy(np.stack([p[0] for p in pairs])).to(dev)
    I1 = torch.from_numpy(np.stack([p[1] for p in pairs])).to(dev)
    del pairs
    if in_dtype == "f16":  # integer-valued 0..255: exact in fp16
        I0, I1 = I0.half(), I1.half()
    u = torch.empty((batch, rows, cols), dtype=torch.float32, device=dev)
    v = torch.empty_like(u)
    ws = hsflow.alloc_workspace(rows, cols, batch, dev)
    pws = (torch.empty(hsflow.pyramid_workspace_bytes(rows, cols, batch, levels),
                       dtype=torch.uint8, device=dev) if levels > 1 else None)
    stream = torch.cuda.current_stream(dev)

    def solve(s):
        if levels > 1:
            hsflow.flow_pyramid_device(I0, I1, levels, args.window, iters, args.alpha, u, v,
                                       pws, s)
        else:
            hsflow.flow_device(I0, I1, args.window, iters, args.alpha, u, v, ws, s)

    # A step is one full solve.  By default it is captured once into a
    # hipGraph (the *_device entry points are stream-ordered and never
    # synchronise or allocate; tests/test_gpu_parity.py checks replay ==
    # eager bit for bit) and replayed, so the host does not have to enqueue
    # the ~100 launches/events of a solve while the GPU waits.
    graph = None
    if not args.no_graph:
        try:
            cap = torch.cuda.Stream(dev)
            cap.wait_stream(stream)
            with torch.cuda.stream(cap):
                solve(cap)  # eager once: the library's side streams exist before capture
            stream.wait_stream(cap)
            torch.cuda.synchronize(dev)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                solve(torch.cuda.current_stream(dev))
            torch.cuda.synchronize(dev)
        except Exception as e:  # pragma: no cover - eager fallback, reported
            print(f"bench: graph capture failed ({e}); timing eager solves", file=sys.stderr)
            graph = None

    def step():
        if graph is not None:
            graph.replay()
        else:
            solve(stream)

    # the process group comes up after the capture: no communicator thread
    # touches the device while a stream is capturing
    init_dist()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()

    px = rows * cols
    # pixels swept per iteration, summed over the pyramid levels
    px_all = sum(r * c for r, c in (hsflow.pyramid_level_size(rows, cols, l)
                                    for l in range(levels)))
    total_pairs = batch * world * args.steps
    value = total_pairs * px_all * iters / elapsed / 1e6
    ok = bool(torch.isfinite(u).all().item()) and 0.05 < float(u.mean()) < 0.3

    # ---- dominant-kernel roofline: K2 alone, events on the launch stream --
    kb = hsflow.iters_per_launch(rows, cols, batch, args.window) if not args.kb else args.kb
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    hsflow.gradients_device(I0, I1, ws, stream=stream)
    launches_per_solve = -(-iters // kb)
    reps = args.roofline_reps
    # one stream here so the per-launch duration is what rocprofv3 reports
    # per dispatch (the batch split overlaps launches and would blur it)
    hsflow.set_max_streams(1)
    torch.cuda.synchronize(dev)
    ev0.record(stream)
    for _ in range(reps):
        hsflow.jacobi_device(rows, cols, batch, args.window, iters, args.alpha, u, v, ws,
                             stream=stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    hsflow.set_max_streams(0)
    k2_ms = ev0.elapsed_time(ev1) / (reps * launches_per_solve)
    n_px = batch * px
    # algorithmic bytes = 28 B per pixel-iteration (read u, v,
    # Ix, Iy, It; write u', v' in f32) x the pixel-iterations one launch
    # performs -- fixed by the algorithm, whatever the blocking saves
    px_iters_per_launch = n_px * iters / launches_per_solve
    bytes_per_launch = 28.0 * px_iters_per_launch
    achieved = bytes_per_launch / (k2_ms * 1e-3) / 1e9
    # the HBM bytes one temporally-blocked pass cannot avoid (what the PMC
    # traffic is compared with): read u, v (f32) + packed gradients (4 B),
    # write u, v; the first pass of a solve reads no u, v
    first_frac = 1.0 / launches_per_solve
    compulsory = n_px * (8 + 4 + 8 - 8 * first_frac)
    compulsory_gbps = compulsory / (k2_ms * 1e-3) / 1e9

    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_{args.workload}.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f)
        if pmc.get("kb") == kb and pmc.get("batch") == batch:
            traffic = pmc.get("hbm_bytes_per_launch")

    cpu = cpu_all = None
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(rows, cols, args.window, args.alpha, args.cpu_iters)
        # SURVEY §8(d) second CPU line: all cores of the box's CPU share
        # (16 per GPU on the MI355X pool; os.cpu_count() shows the machine)
        n_thr = min(16, os.cpu_count() or 1)
        cpu_all = cpu_baseline(rows, cols, args.window, args.alpha, args.cpu_iters, n_thr)

    if rank == 0:
        line = {
            "metric": "Mpix*iter/s (Horn-Schunck Jacobi) + frame-pairs/s",
            "value": round(value, 1),
            "unit": "Mpix*iter/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic {in_dtype} frame pairs (hash texture, shift (-0.75,+1.5) px)",
            "config": {"workload": f"{args.workload} {cols}x{rows}, {iters} it"
                                   + (f"/level x {levels} levels" if levels > 1 else "")
                                   + f", ws {args.window}",
                       "rows": rows, "cols": cols, "iters": iters, "window": args.window,
                       "levels": levels, "input_dtype": in_dtype,
                       "alpha": args.alpha, "pairs_per_gpu_per_step": batch,
                       "iters_per_launch": kb, "parallelism": f"frame-parallel x{world}",
                       "step": "hipGraph replay of one solve" if graph is not None
                               else "eager solve"},
            "pairs_per_s": round(total_pairs / elapsed, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic,
                         "kernel": "hs_jacobi_wg_kernel",
                         "avg_launch_ms": round(k2_ms, 5),
                         "iters_per_launch": kb,
                         "algorithmic_bytes_per_launch": int(bytes_per_launch),
                         "algorithmic_B_per_px_iter": 28,
                         "compulsory_bytes_per_launch": int(compulsory),
                         "compulsory_GBps": round(compulsory_gbps, 1),
                         "compulsory_frac": round(compulsory_gbps / HBM_PEAK_GBPS, 4),
                         # measured (DESIGN.md §4 Roofline): the pass is bound
                         # by VALU issue, its compute phase at ~95 % of the
                         # wave64 VALU rate; HBM is the nominal SURVEY class
                         "limiter": "valu"},
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_all,
            "sane": ok,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def stream_mode(args, world, rank, dev):
    """BASELINE config 4: a stream of --pairs synthetic frame pairs held by
    rank 0, scattered one-per-rank round-robin over RCCL (point-to-point),
    solved (each rank batches its share into one hsflow_flow_device call),
    and (u, v) gathered back to rank 0.  Timed end to end (scatter + solve +
    gather), max over ranks.  Reported as pairs/s and Mpix*iter/s."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import hsflow
    import frame_parallel as fp

    wl = dict(WORKLOADS[args.workload])
    rows, cols = wl["rows"], wl["cols"]
    iters = args.iters or wl["iters"]
    n = args.pairs
    stream = None
    if rank == 0:
        stream = [tuple(torch.from_numpy(a).to(dev) for a in
                        hsflow.synth_pair(1000 + j, rows, cols)) for j in range(n)]
    mine = fp.my_pairs(n, rank, world)
    ws = hsflow.alloc_workspace(rows, cols, max(1, len(mine)), dev)

    def one_pass():
        pairs = fp.scatter_pairs(stream, n, (rows, cols), torch.float32, dev, rank, world)
        flows = []
        if pairs:
            I0 = torch.stack([p[0] for p in pairs])
            I1 = torch.stack([p[1] for p in pairs])
            u, v = hsflow.flow_device(I0, I1, args.window, iters, args.alpha, workspace=ws)
            flows = [(u[k], v[k]) for k in range(len(pairs))]
        return fp.gather_flows(flows, n, (rows, cols), dev, rank, world)

    for _ in range(args.warmup):
        one_pass()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = one_pass()
    torch.cuda.synchronize(dev)
    elapsed = fp.max_over_ranks(time.perf_counter() - t0, dev, world)
    if rank == 0:
        ok = len(out) == n and all(bool(torch.isfinite(u).all()) for u, _ in out[:2])
        total = n * args.steps
        print(json.dumps({
            "metric": "frame-pairs/s (config 4 stream: RCCL scatter + solve + gather)",
            "value": round(total / elapsed, 2), "unit": "pairs/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic f32 frame pairs",
            "config": {"workload": f"stream of {n} x {args.workload} pairs, {iters} it",
                       "pairs": n, "iters": iters, "window": args.window,
                       "parallelism": f"frame-parallel x{world}"},
            "Mpix_iter_per_s": round(total * rows * cols * iters / elapsed / 1e6, 1),
            "sane": ok}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bands_mode(args, world, rank, dev):
    """BASELINE config 5 across ranks: one pair (default the 8k workload,
    fp16, 3 levels) split into row bands; every `--chunk` iterations each
    rank exchanges halo rows with its neighbours over RCCL, and rank 0
    gathers (u, v).  Timed: pyramid build + banded levels + exchanges +
    gather (inputs broadcast from rank 0 beforehand, resident in HBM).
    Strong scaling: the work is fixed, value = pair Mpix*iter/s."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import hsflow
    import row_bands as rb

    wl = dict(WORKLOADS[args.workload if args.workload != "1080p" else "8k"])
    rows, cols = wl["rows"], wl["cols"]
    iters = args.iters or wl["iters"]
    levels = args.levels or wl.get("levels", 1)
    in_dtype = args.dtype or wl.get("dtype", "f32")
    tdt = {"f16": torch.float16, "f32": torch.float32, "u8": torch.uint8}[in_dtype]
    I0 = torch.empty((rows, cols), dtype=tdt, device=dev)
    I1 = torch.empty_like(I0)
    if rank == 0:
        a, b = hsflow.synth_pair(1000, rows, cols,
                                 dtype=np.uint8 if in_dtype == "u8" else np.float32)
        I0.copy_(torch.from_numpy(a).to(dev).to(tdt))
        I1.copy_(torch.from_numpy(b).to(dev).to(tdt))
    if world > 1:
        dist.broadcast(I0, 0)
        dist.broadcast(I1, 0)
    p = rb.plan(rows, cols, levels, world, args.window, args.chunk)
    ops = [rb.DeviceOps(args.window, args.alpha, dev)]
    comm = rb.DistComm() if world > 1 else rb.LocalComm()

    def one():
        states = rb.solve([I0], [I1], p, iters, ops, comm, [rank])
        return rb.gather_owned(states, p, comm)

    for _ in range(args.warmup):
        one()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        u, v = one()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    px_all = sum(r * c for r, c in p.sizes)
    if rank == 0:
        ok = bool(torch.isfinite(u).all().item()) and 0.05 < float(u.mean()) < 0.3
        print(json.dumps({
            "metric": "Mpix*iter/s (config 5: one pair in row bands, halo exchange over RCCL)",
            "value": round(px_all * iters * args.steps / elapsed / 1e6, 1),
            "unit": "Mpix*iter/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f32", "data": f"synthetic {in_dtype} frame pair",
            "config": {"workload": f"{cols}x{rows}, {levels} levels, {iters} it/level",
                       "window": args.window, "chunk": args.chunk, "halo_rows": p.halo,
                       "parallelism": f"row bands x{world}"},
            "sane": ok}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(rows, cols, window, alpha, cpu_iters, threads=1):
    """oracle/ float64 port of hornSchunck.cpp (pass-per-OpenCV-call, fresh
    temporaries each iteration) on the same synthetic pair at full size for a
    bounded number of iterations; 1 thread like the reference,
    or `threads` OpenMP threads for the all-cores variant."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    import hsflow
    I0, I1 = hsflow.synth_pair(1000, rows, cols)
    if not cpu_iters:
        t = time.perf_counter()
        oracle.flow(I0, I1, window, 1, alpha, nthreads=threads)
        one = time.perf_counter() - t
        cpu_iters = max(1, min(60, int(15.0 / max(one, 1e-3))))
    t = time.perf_counter()
    oracle.flow(I0, I1, window, cpu_iters, alpha, nthreads=threads)
    dt = time.perf_counter() - t
    return {"value": round(rows * cols * cpu_iters / dt / 1e6, 2), "unit": "Mpix*iter/s",
            "cores": threads, "kind": "port",
            "sample": f"{cols}x{rows} pair, {cpu_iters} Jacobi iterations incl. gradients, "
                      f"float64, {dt:.1f} s"}


if __name__ == "__main__":
    main()
