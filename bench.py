"""Horn-Schunck throughput bench (BASELINE.json metric: Mpix*iter/s + pairs/s).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload 1080p|4k|8k]

One step = one full solve (K1 gradients + `iters` Jacobi iterations, the
reference's getFlow, hornSchunck.cpp:43-75) of a batch of synthetic frame
pairs per GPU, inputs already resident in HBM (workload 8k = BASELINE config
5: an fp16 7680x4320 pair through the 3-level coarse-to-fine warm start,
`iters` per level; its Mpix*iter counts every level's pixels).  Frame pairs
are independent, so for N > 1 each rank (one process per GPU,
torch.distributed over RCCL) solves its own pairs: weak scaling, no
data-path collective (the timing barrier and max-over-ranks reduction are
the only collectives in the headline leg).

`--gpus N` is authoritative: without a launcher (no WORLD_SIZE in the
environment) and N > 1, bench.py starts N rank processes itself
(torch.distributed.run, 127.0.0.1) and exits with their status; under a
launcher whose WORLD_SIZE differs from N it refuses to run (status 2).

Rank 0 prints ONE JSON line.  Every timed output is checked: before the
timed steps the output planes are filled with NaN, so a pass only if the
timed replays themselves computed (u, v); a parity miss anywhere exits 3.
  parity        pair 0 of the TIMED solve (seed 1000) against the float64
                oracle's golden checksums (tests/golden/bench_golden.*,
                made by tests/golden/make_bench_golden.py): max|du|/max|u| on
                a strided sample and the whole-plane sums
  parity_all    one verdict per BASELINE config: configs[0] (KITTI crop,
                host API), [1] (1080p x 300, batched and single pair), [2]
                (4K x 500, batched and single pair), [3] (the stream of 64
                pairs: pair 0 vs the golden, pairs 0..7 bit for bit against
                the resident solve of the same seeds), [4] (8K fp16, 3 levels
                x 1000 it)
  roofline      the dominant kernel, the Jacobi pass (`kernel`: K4
                hs_jacobi_strip_kernel or K2 hs_jacobi_wg_kernel, whichever
                the library runs for the leg).  The top-level figures
                describe the TIMED step: avg_launch_ms = ms_per_step / passes
                per solve (the wall time of one pass of the whole batch, both
                side streams, K1's share included -- so the kernel's time per
                step never exceeds ms_per_step); achieved = the algorithmic
                bytes of one temporally blocked pass (read u, v and the
                packed gradients, write u, v: 20 B per pixel; the first pass
                reads no u, v) / avg_launch_ms, frac = achieved / 8 TB/s (a
                physical fraction, <= 1); traffic = PMC bytes per pass of the
                timed configuration (profiles/pmc_r06.json, rocprofv3 --pmc of
                scripts/timed_step.py), hbm_frac = traffic / avg_launch_ms /
                8 TB/s.  `isolated_launch`: one single-stream launch timed
                with events on its stream (what rocprofv3 reports per
                dispatch), with its own PMC bytes and VALU issue fractions;
                naive_equiv_frac = SURVEY §8(d)'s 28 B per pixel-iteration x
                the iterations one launch performs / launch time / 8 TB/s
                (the rate a one-iteration-per-launch kernel would need;
                exceeds 1 by design, DESIGN.md "Roofline")
  secondary     BASELINE configs[2] (4K x 2 pairs x 500 it)
  config5       BASELINE configs[4] (8K fp16, 3-level pyramid, 1000 it/level)
  single_pair   configs[1] and configs[2] as stated: ONE pair per solve
                (the reference's call pattern, main.cpp:97-98)
  window3       north_star's windowSize 3 on the 1080p batch
  pairs_per_s_resident / pairs_per_s_e2e
                pairs/s with inputs in HBM, and end to end as BASELINE.md
                defines it: pinned host u8 frames -> H2D -> K1 + K2 -> D2H
                of (u, v) f32, copies overlapped with solves on other streams
  stream        BASELINE config 4: 64 pairs held by rank 0, scattered over
                RCCL (point-to-point), solved, (u, v) gathered back, checked
  bands         BASELINE config 5 as stated for N GPUs: ONE 8K fp16 pair
                (3 levels x 1000 it) split into N row bands with a halo
                exchange over RCCL (row_bands.solve), checked against the
                8k_w5_l3 golden; at N = 1 one band (the config5 leg's solve
                through the band machinery)
  host_api      the reference's own call (main.cpp:97-98): one pair through
                hsflow_flow from pageable host u8 frames to CV_64FC1 (u, v)
                (hornSchunck.cpp:49-50, 72-73), 1080p and 4K, with parity
  cpu_baseline  the float64 CPU port (oracle/, mirrors hornSchunck.cpp pass
                by pass) on a bounded sample, 1 thread, rank 0 (also on N > 1
                lines: the host-core figure next to every GPU count)
"""
from __future__ import annotations

import argparse
import json
import mmap
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))

WORKLOADS = {
    # BASELINE.json configs[1] / configs[2]
    "1080p": dict(rows=1080, cols=1920, iters=300, batch=8),
    "4k": dict(rows=2160, cols=3840, iters=500, batch=2),
    # BASELINE.json configs[4] on one GPU (the 8-GPU row-band split is
    # --mode bands; frame-parallel weak scaling is the headline)
    "8k": dict(rows=4320, cols=7680, iters=1000, batch=1, levels=3, dtype="f16"),
}
HBM_PEAK_GBPS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
COPY_PEAK_GBPS = 6290.0    # MI355X_MICROARCH.md: float4 copy, measured (79 % of spec)
PASS_BYTES_PER_PX = 20     # one blocked pass: read u, v (8) + packed gradients (4),
                           # write u, v (8); DESIGN.md "Roofline"
NAIVE_BYTES_PER_PX_ITER = 28  # f32 u, v, Ix, Iy, It in, u', v' out
PARITY_TOL = 1e-4          # north_star: 1e-4 relative (norm form)
GOLDEN_JSON = os.path.join(ROOT, "tests", "golden", "bench_golden.json")
GOLDEN_NPZ = os.path.join(ROOT, "tests", "golden", "bench_golden.npz")
PMC_JSON = os.path.join(ROOT, "profiles", "pmc_r06.json")
# bands leg: coarse levels up to this many pixels are solved whole on every
# rank (the 8K pyramid's 1920 x 1080 level 2; row_bands.whole_levels)
BANDS_WHOLE_MAX_PX = 2_200_000
# iterations between exchanges per level for the 2-D block split (N = 8
# predicted 14.4 ms per 8K pair at 48,96 against 23.6 at 24,48: the
# exchange's fixed cost dominates a 24-iteration chunk of a 2256 x 2112
# block; profiles/r06_blocks_prediction.json)
BLOCKS_CHUNK = "48,96"
ROWS_CHUNK = "24,48"
# (relative to csrc/; the Makefile carries the per-file scheduler flags)
KERNEL_SOURCES = ("hsflow_strips.hip", "hsflow_kernels.hip", "hsflow_device.h", "../Makefile")
# measured VALU issue cost per wave64 instruction per SIMD (shader cycles)
# at each Jacobi kernel's occupancy: profiles/r02_valu_tput.txt, mean of
# v_add / v_add_dpp / v_pk_add / v_fma / v_pk_fma at 2 (K4) and 4 (K2)
# waves per SIMD
ISSUE_CYCLES = {"hs_jacobi_strip_kernel": 4.84, "hs_jacobi_wg_kernel": 3.32}
# HSFLOW_* variables the bench itself reads (rehearsal of the N > 1 logic
# with several ranks on one GPU); every other HSFLOW_* name is refused
BENCH_ENV = {"HSFLOW_BENCH_BACKEND", "HSFLOW_BENCH_DEVICE"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs = ranks; without a launcher bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
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
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the configs[2] (4K) block of the default run")
    ap.add_argument("--no-w3", action="store_true",
                    help="skip the window-3 block of the default run (SURVEY §8d)")
    ap.add_argument("--no-8k", action="store_true",
                    help="skip the configs[4] (8K pyramid) block of the default run")
    ap.add_argument("--no-single", action="store_true",
                    help="skip the single-pair blocks of the default run")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end pairs/s leg")
    ap.add_argument("--no-stream", action="store_true", help="skip the config-4 stream leg")
    ap.add_argument("--no-bands", action="store_true",
                    help="skip the config-5 row-band leg of the default run")
    ap.add_argument("--no-host-api", action="store_true",
                    help="skip the host-buffer getFlow leg of the default run")
    ap.add_argument("--mode", choices=["resident", "stream", "bands"], default="resident",
                    help="resident: pairs generated on each rank, already in HBM "
                         "(the metric, plus the secondary / e2e / stream legs); stream: "
                         "BASELINE config 4 alone; bands: BASELINE config 5 on N GPUs, "
                         "ONE pair split into row bands with a halo exchange")
    ap.add_argument("--chunk", default=None,
                    help="bands: iterations between halo exchanges, one value or one per "
                         "pyramid level from the finest (the last repeats): coarse levels "
                         "carry little work per chunk, so longer chunks there save "
                         "exchanges (default 48,96 for blocks, 24,48 for row bands)")
    ap.add_argument("--split", choices=["auto", "rows", "blocks"], default="auto",
                    help="bands: how one pair is split over N ranks: row bands "
                         "(row_bands.py) or a 2-D grid of blocks (blocks.py); auto = "
                         "blocks (fewer halo pixels and bytes per exchange; "
                         "scripts/scale_predict.py --blocks), rows with --overlap")
    ap.add_argument("--overlap", action="store_true",
                    help="bands mode: hide each exchange behind the next chunk's interior "
                         "(row_bands.solve_overlapped; bit-identical)")
    ap.add_argument("--pairs", type=int, default=64, help="stream leg: pairs in the stream")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks, check they see each other (gloo all-reduce), "
                         "print n_gpus and exit: the launcher plumbing alone, no GPU work")
    return ap.parse_args(argv)


# --------------------------------------------------------------- guards
def refuse_diagnostics(environ=None):
    """Names of HSFLOW_* variables set in the environment other than the
    bench's own.  The library reads none, but hsflow.py honours HSFLOW_LIB
    (another build of the library, for same-box A/B): the bench refuses them
    all so a stray variable can never produce a number."""
    environ = os.environ if environ is None else environ
    return sorted(k for k in environ if k.startswith("HSFLOW_") and k not in BENCH_ENV)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def world_from_env(gpus, environ=None):
    """(action, world): ("launch", N) when N > 1 ranks must be started here
    (no launcher), ("run", world) under a launcher that agrees with --gpus or
    for one GPU, ("refuse", world) when WORLD_SIZE contradicts --gpus."""
    environ = os.environ if environ is None else environ
    ws = environ.get("WORLD_SIZE")
    if ws is None:
        return ("launch", gpus) if gpus > 1 else ("run", 1)
    world = int(ws)
    return ("run", world) if world == gpus else ("refuse", world)


def launch_ranks(n):
    """One process per GPU, started the way the driver starts them
    (torch.distributed.run, one node, 127.0.0.1).  A child process, not an
    exec: nothing in this process has touched the GPU.  Rank 0's stdout is
    this process's stdout (the one JSON line)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def launch_check(world, rank):
    """--launch-check: every rank joins a gloo group and all-reduces a one;
    rank 0 prints what it saw.  No GPU work (CPU-testable)."""
    import torch
    import torch.distributed as dist
    seen = 1
    if world > 1:
        dist.init_process_group("gloo")
        t = torch.ones(1)
        dist.all_reduce(t)
        seen = int(t.item())
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks_seen": seen,
                          "launcher": "torch.distributed.run" if world > 1 else "none"}),
              flush=True)
    return 0 if seen == world else 4


# --------------------------------------------------------------- parity
def golden_entry(rows, cols, iters, window, levels, alpha):
    """(name, meta, u_sample, v_sample) of the committed oracle golden for
    this configuration, or None."""
    import numpy as np
    if not (os.path.exists(GOLDEN_JSON) and os.path.exists(GOLDEN_NPZ)):
        return None
    meta = json.load(open(GOLDEN_JSON))
    for name, e in meta.items():
        if (e["rows"], e["cols"], e["iters"], e["window"], e["levels"], e["alpha"]) == \
                (rows, cols, iters, window, levels, alpha):
            z = np.load(GOLDEN_NPZ)
            return name, e, z[name + "_u"], z[name + "_v"]
    return None


def parity_check(u, v, golden):
    """u, v: full float planes (numpy) of pair seed 1000.  Compares the
    strided sample elementwise (max|d| / max|ref|, the SURVEY §8c form, scale
    = the oracle's full-plane max) and the plane sums (|dSum| / (n max|ref|))."""
    import numpy as np
    if golden is None:
        return {"ok": None, "reason": "no golden for this configuration"}
    name, e, us, vs = golden
    step = e["step"]
    n = u.size
    out = {"golden": name, "tol": PARITY_TOL}
    errs, sums = [], []
    for got, ref, s_ref, m_ref in ((u, us, e["sum_u"], e["max_u"]),
                                   (v, vs, e["sum_v"], e["max_v"])):
        g = np.asarray(got, np.float64)
        errs.append(float(np.max(np.abs(g[::step, ::step] - ref))) / m_ref)
        sums.append(abs(float(g.sum()) - s_ref) / (n * m_ref))
    out["max_rel_err"] = max(errs)
    out["sum_rel_err"] = max(sums)
    out["ok"] = bool(np.isfinite(u).all() and np.isfinite(v).all() and
                     out["max_rel_err"] <= PARITY_TOL and out["sum_rel_err"] <= PARITY_TOL)
    return out


# --------------------------------------------------------------- timing
PREWARM_S = 0.15
_T0 = time.perf_counter()


def progress(msg, rank=0):
    """One stderr line per leg (the GPU pool takes a command that prints
    nothing for 3 minutes for hung); stdout keeps the one JSON line."""
    print(f"bench [rank {rank}, {time.perf_counter() - _T0:6.1f} s]: {msg}", file=sys.stderr,
          flush=True)


def prewarm(step, sync, seconds=PREWARM_S, max_steps=400):
    """Untimed steps until `seconds` of load have passed, before the W
    warm-up steps: the GPU needs ~0.1 s under load to reach its steady
    clocks (same box, 1080p x 8: 2 warm-up steps read 1.22-1.24 M, 20 read
    1.33 M, 60 1.34 M; profiles/HISTORY.md), so a short driver warm-up would time
    the clock ramp, not the kernels.  Returns (steps, seconds) run."""
    sync()
    t0 = time.perf_counter()
    n = 0
    while n < max_steps:
        step()
        n += 1
        if n % 4 == 0 or n == 1:
            sync()
            if time.perf_counter() - t0 >= seconds:
                break
    sync()
    return n, time.perf_counter() - t0


def timed_region(step, sync, steps, warmup, world, device, info=None, prewarm_s=0.0,
                 before_timing=None):
    """The driver's timing rule: W untimed steps, barrier + sync, K timed
    steps, sync; the slowest rank's time.  With prewarm_s > 0, `prewarm`
    runs first (untimed; what it ran goes into `info`) -- only for steps
    without collectives: a time-bounded loop may run different step counts
    on different ranks."""
    import torch
    import torch.distributed as dist
    if prewarm_s > 0:
        n, t = prewarm(step, sync, prewarm_s)
        if info is not None:
            info["prewarm_steps"] = n
            info["prewarm_s"] = round(t, 3)
    for _ in range(warmup):
        step()
    if before_timing is not None:
        before_timing()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    return elapsed


def pmc_key(wl_name, window, batch):
    return f"{wl_name}_w{window}_b{batch}"


def kernel_source_md5():
    """md5 of the Jacobi kernels' sources: a committed PMC profile is used
    only for the kernel code it was collected on"""
    import hashlib
    h = hashlib.md5()
    for name in KERNEL_SOURCES:
        with open(os.path.join(ROOT, "cpp-optical-flow_amd", "csrc", name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def pmc_for(wl_name, window, batch, kb, kernel, timed=False, passes=None):
    """Committed PMC summary of this roofline leg (profiles/pmc_r06.json,
    written by scripts/pmc_collect.py from separate rocprofv3 --pmc passes)
    if it was collected for this kernel, blocking depth, batch and kernel
    source.  timed: the timed configuration's entry (scripts/timed_step.py:
    the bench's graph-replayed solve on its side streams) instead of the
    single-stream launches."""
    if not os.path.exists(PMC_JSON):
        return None
    with open(PMC_JSON) as f:
        e = json.load(f).get(("step_" if timed else "") + pmc_key(wl_name, window, batch))
    if e and e.get("kb") == kb and e.get("kernel") == kernel and \
            e.get("kernel_source_md5") == kernel_source_md5() and \
            (passes is None or e.get("passes_per_solve") == passes):
        return e
    return None


def roofline_leg(wl_name, hsflow, dev, I0, I1, rows, cols, batch, window, iters, alpha,
                 reps, step_ms=None, ws=None):
    """Roofline of the dominant kernel, the Jacobi pass (K4 or K2, as the
    library picks for the leg).  Top level: the TIMED step (step_ms =
    ms_per_step of the leg): one pass of the whole batch takes step_ms /
    passes of wall time.  `isolated_launch`: one single-stream launch timed
    with events on its stream -- the per-dispatch duration rocprofv3
    reports.  Config 5: the level-0 plane, the pass that dominates its solve."""
    import torch
    kb = hsflow.iters_per_launch(rows, cols, batch, window)
    kernel = hsflow.jacobi_kernel_name(rows, cols, batch, window)
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    rws = ws if ws is not None else hsflow.alloc_workspace(rows, cols, batch, dev)
    u = torch.empty((batch, rows, cols), dtype=torch.float32, device=dev)
    v = torch.empty_like(u)
    hsflow.gradients_device(I0, I1, rws, stream=stream)
    launches_per_solve = -(-iters // kb)
    # one stream so the per-launch duration is what rocprofv3 reports per
    # dispatch (the batch split overlaps launches and would blur it)
    with hsflow.max_streams_as(1):
        hsflow.jacobi_device(rows, cols, batch, window, iters, alpha, u, v, rws, stream=stream)
        torch.cuda.synchronize(dev)
        ev0.record(stream)
        for _ in range(reps):
            hsflow.jacobi_device(rows, cols, batch, window, iters, alpha, u, v, rws,
                                 stream=stream)
        ev1.record(stream)
        torch.cuda.synchronize(dev)
    k2_ms = ev0.elapsed_time(ev1) / (reps * launches_per_solve)
    n_px = batch * rows * cols
    # algorithmic bytes of one blocked pass: u, v in (the first pass of a
    # solve reads none), packed gradients in, u, v out
    pass_bytes = n_px * (PASS_BYTES_PER_PX - 8 / launches_per_solve)
    achieved = pass_bytes / (k2_ms * 1e-3) / 1e9
    naive = NAIVE_BYTES_PER_PX_ITER * n_px * iters / launches_per_solve / (k2_ms * 1e-3) / 1e9
    iso = {"avg_launch_ms": round(k2_ms, 5), "achieved": round(achieved, 1),
           "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None,
           "naive_equiv_frac": round(naive / HBM_PEAK_GBPS, 4),
           "naive_B_per_px_iter": NAIVE_BYTES_PER_PX_ITER,
           "hbm_frac": None, "valu_frac": None, "valu_issue_frac": None,
           "timing": "single stream, events on the launch stream"}
    pmc = pmc_for(wl_name, window, batch, kb, kernel)
    if pmc is not None and pmc.get("hbm_bytes_per_launch"):
        traffic = pmc["hbm_bytes_per_launch"]
        iso["traffic"] = traffic
        iso["traffic_over_algorithmic"] = round(traffic / pass_bytes, 3)
        # physical HBM utilisation: the PMC bytes at the live launch time
        iso["hbm_frac"] = round(traffic / (k2_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
        iso["hbm_frac_vs_copy_peak"] = round(
            traffic / (k2_ms * 1e-3) / 1e9 / COPY_PEAK_GBPS, 4)
        if pmc.get("valu_insts_per_launch") and pmc.get("launch_cycles"):
            # VALU issue at the guide's 2 cycles per wave64 instruction per
            # SIMD (MI355X_MICROARCH.md constants table) over the launch's
            # shader cycles (GRBM_GUI_ACTIVE / 8 XCDs)
            iso["valu_frac"] = round(pmc["valu_insts_per_launch"] * 2.0 / 1024 /
                                     pmc["launch_cycles"], 4)
            if kernel in ISSUE_CYCLES:
                # the same at the issue rate the kernel's occupancy allows
                iso["valu_issue_frac"] = round(
                    pmc["valu_insts_per_launch"] * ISSUE_CYCLES[kernel] / 1024 /
                    pmc["launch_cycles"], 4)
            iso["clock_ghz"] = pmc.get("clock_ghz")
        iso["pmc_source"] = pmc.get("source")
    # the timed step: one pass of the whole batch per step_ms / passes
    pass_ms = step_ms / launches_per_solve if step_ms else k2_ms
    ach = pass_bytes / (pass_ms * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS,
            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": None,
            "kernel": kernel, "avg_launch_ms": round(pass_ms, 5),
            "timing": ("timed step: ms_per_step / passes per solve (hipGraph replay, "
                       "batch split over the side streams; K1 included)") if step_ms
                      else "isolated launch",
            "iters_per_launch": kb, "launches_per_solve": launches_per_solve,
            "algorithmic_bytes_per_launch": int(pass_bytes),
            "algorithmic_B_per_px_pass": PASS_BYTES_PER_PX, "hbm_frac": None,
            "naive_equiv_frac": round(NAIVE_BYTES_PER_PX_ITER * n_px * iters /
                                      launches_per_solve / (pass_ms * 1e-3) / 1e9 /
                                      HBM_PEAK_GBPS, 4),
            "isolated_launch": iso}
    tp = (pmc_for(wl_name, window, batch, kb, kernel, timed=True, passes=launches_per_solve)
          if step_ms else None)
    if tp is not None and tp.get("hbm_bytes_per_step"):
        per_pass = tp["hbm_bytes_per_step"] / launches_per_solve
        roof["traffic"] = int(per_pass)
        roof["traffic_over_algorithmic"] = round(per_pass / pass_bytes, 3)
        roof["hbm_frac"] = round(per_pass / (pass_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
        roof["traffic_source"] = tp.get("source")
    elif iso["traffic"] is not None:
        # no profile of the timed configuration: the isolated launch's bytes
        roof["traffic"] = iso["traffic"]
        roof["traffic_over_algorithmic"] = iso["traffic_over_algorithmic"]
        roof["hbm_frac"] = round(iso["traffic"] / (pass_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
        roof["traffic_source"] = "isolated launch PMC bytes (" + str(iso.get("pmc_source")) + ")"
    del u, v
    return roof


# --------------------------------------------------------------- resident
def resident_leg(wl_name, args, dev, world, rank, init_dist=None, window=None, batch=None,
                 keep=False, roofline=True):
    """One workload, inputs resident in HBM: a step is one full solve of
    `batch` pairs per rank (hipGraph replay).  Returns the leg's dict (and,
    with keep, rank 0's timed (u, v) for cross-checks)."""
    import numpy as np
    import torch
    import hsflow

    wl = dict(WORKLOADS[wl_name])
    rows, cols = wl["rows"], wl["cols"]
    iters = args.iters or wl["iters"]
    batch = batch or args.batch or wl["batch"]
    levels = args.levels or wl.get("levels", 1)
    in_dtype = args.dtype or wl.get("dtype", "f32")
    window, alpha = (window or args.window), args.alpha

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
            hsflow.flow_pyramid_device(I0, I1, levels, window, iters, alpha, u, v, pws, s)
        else:
            hsflow.flow_device(I0, I1, window, iters, alpha, u, v, ws, s)

    # A step is one full solve, captured once into a hipGraph and replayed
    # (the *_device entry points are stream-ordered and never synchronise or
    # allocate; tests/test_gpu_parity.py checks replay == eager bit for bit).
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
            # thread_local: only this thread's calls can invalidate the
            # capture (the secondary leg captures after the process group,
            # whose watchdog thread polls events, is up)
            # the capture's origin stream calls the library itself, so the
            # batch split (automatic: off under capture) is safe to ask for
            with hsflow.max_streams_as(2), \
                    torch.cuda.graph(graph, capture_error_mode="thread_local"):
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

    # the output planes hold NaN when the timed steps start (filled after
    # the pre-warm and warm-up replays): the parity check below passes only
    # if the timed replays themselves wrote (u, v)
    def nan_fill():
        u.fill_(float("nan"))
        v.fill_(float("nan"))
    nan_fill()
    torch.cuda.synchronize(dev)
    # the process group comes up after the first capture: no communicator
    # thread touches the device while a stream is capturing
    if init_dist is not None:
        init_dist()
    warm = {}
    elapsed = timed_region(step, lambda: torch.cuda.synchronize(dev), args.steps,
                           args.warmup, world, dev, info=warm, prewarm_s=PREWARM_S,
                           before_timing=nan_fill)

    # parity of the timed output: pair 0 of rank 0 is seed 1000
    parity = None
    if rank == 0:
        golden = golden_entry(rows, cols, iters, window, levels, alpha)
        parity = parity_check(u[0].cpu().numpy(), v[0].cpu().numpy(), golden)
        parity["outputs_nan_filled_before_timing"] = True
    kept = (u.clone(), v.clone()) if (keep and rank == 0) else None

    px_all = sum(r * c for r, c in (hsflow.pyramid_level_size(rows, cols, l)
                                    for l in range(levels)))
    total_pairs = batch * world * args.steps
    value = total_pairs * px_all * iters / elapsed / 1e6

    step_kind = "hipGraph replay of one solve" if graph is not None else "eager solve"
    del u, v, graph
    roof = None
    if roofline:
        # config 5: the level-0 plane's passes are most of the step, not all
        roof = roofline_leg(wl_name, hsflow, dev, I0, I1, rows, cols, batch, window, iters,
                            alpha, args.roofline_reps,
                            step_ms=elapsed / args.steps * 1e3 if levels == 1 else None,
                            ws=ws if levels == 1 else None)

    leg = {"workload": f"{wl_name} {cols}x{rows}, {iters} it"
                       + (f"/level x {levels} levels" if levels > 1 else "")
                       + f", ws {window}" + (f", {batch} pair" + ("s" if batch > 1 else "")),
           "rows": rows, "cols": cols, "iters": iters, "window": window, "levels": levels,
           "input_dtype": in_dtype, "alpha": alpha, "pairs_per_gpu_per_step": batch,
           "value": round(value, 1), "unit": "Mpix*iter/s",
           "ms_per_step": round(elapsed / args.steps * 1e3, 3),
           "pairs_per_s_resident": round(total_pairs / elapsed, 2),
           "step": step_kind, "untimed_prewarm": warm, "roofline": roof, "parity": parity}
    del I0, I1, ws, pws
    torch.cuda.empty_cache()
    if keep:
        return leg, kept
    return leg


def hbm_stream_peak(dev, nbytes=2 << 30, reps=5):
    """Measured device copy rate (read + write bytes per second, GB/s) of a
    2 GiB buffer, far past the 256 MB Infinity Cache: the practical HBM
    ceiling the roofline is also quoted against."""
    import torch
    n = nbytes // 4
    a = torch.empty(n, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    a.fill_(1.0)
    b.copy_(a)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize(dev)
    gbps = 2 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    torch.cuda.empty_cache()
    return round(gbps, 1)


def config1_leg(dev, reps=20):
    """BASELINE configs[0]: the KITTI 000050 centre
    crop, 256x256 u8, ws 5, alpha 1, 100 iterations -- the reference's own
    CPU-runnable case.  GPU: the host-buffer getFlow path (hsflow_flow:
    upload, solve, CV_64FC1 download), median of `reps`; parity against the
    committed golden (u, v) of the crop (tests/golden/crop256.npz, pinned by
    the reference's plots); CPU: the float64 port on 1 thread."""
    import numpy as np
    import hsflow
    z = np.load(os.path.join(ROOT, "tests", "golden", "crop256.npz"))
    I0, I1 = z["I0"], z["I1"]
    hs = hsflow.hornSchunck(5, 100, 1.0)
    u, v = hs.getFlow(I0, I1)  # warm
    ts = []
    for _ in range(reps):
        u.fill(np.nan)
        v.fill(np.nan)
        t = time.perf_counter()
        u, v = hs.getFlow(I0, I1)
        ts.append(time.perf_counter() - t)
    ms = sorted(ts)[len(ts) // 2] * 1e3
    err = max(float(np.max(np.abs(u - z["u"]))) / float(np.max(np.abs(z["u"]))),
              float(np.max(np.abs(v - z["v"]))) / float(np.max(np.abs(z["v"]))))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    t = time.perf_counter()
    oracle.flow(I0.astype(np.float64), I1.astype(np.float64), 5, 100, 1.0, nthreads=1)
    cpu_ms = (time.perf_counter() - t) * 1e3
    ok = bool(np.isfinite(u).all() and np.isfinite(v).all() and err <= PARITY_TOL)
    return {"workload": "KITTI 000050 crop 256x256 u8, ws 5, alpha 1, 100 it",
            "gpu_ms_host_api": round(ms, 3), "cpu_port_ms_1_thread": round(cpu_ms, 1),
            "parity": {"golden": "crop256", "max_rel_err": err, "ok": ok}}


# --------------------------------------------------------------- e2e
E2E_WARM_S = 0.4


def e2e_leg(wl_name, args, dev, n_batches=48, slots=3):
    """End-to-end pairs/s as BASELINE.md defines it: pinned host u8 gray
    frames (what main.cpp:13-14 hands over) -> H2D -> K1 + K2 -> D2H of u, v
    (f32), batch after batch.  Copies run on their own streams and overlap
    the neighbouring batches' solves (`slots` device buffers in rotation: a
    batch's upload, solve and download each have a slot of their own).  The
    downloads go through hsflow_download_device (the runtime's DMA engines):
    torch's copy_ into pinned memory runs as a 256-workgroup blit kernel per
    plane that takes the next batch's Jacobi workgroup slots (1275 vs ~1600
    pairs/s; scripts/e2e_probe.py, scripts/pcie/d2h_engine_probe.hip).
    A stream of n_batches batches (384 pairs): the pipeline's fill (the
    first upload) and drain (the last 2.4 ms download) are paid once per
    stream, as a video would pay them; with 12 batches they were 10 % of
    the time (rocprofv3 trace of scripts/e2e_probe.py: 4.6 ms per solve with
    the downloads running beside it against 4.3 ms alone, profiles/HISTORY.md)."""
    import numpy as np
    import torch
    import hsflow

    wl = WORKLOADS[wl_name]
    rows, cols, iters, batch = wl["rows"], wl["cols"], args.iters or wl["iters"], wl["batch"]
    host_in = []
    for k in range(2):  # two distinct host batches, alternating
        ps = [hsflow.synth_pair(1000 + 8 * k + i, rows, cols, dtype=np.uint8)
              for i in range(batch)]
        host_in.append((torch.from_numpy(np.stack([p[0] for p in ps])).pin_memory(),
                        torch.from_numpy(np.stack([p[1] for p in ps])).pin_memory()))
    shp = (batch, rows, cols)
    d_in = [(torch.empty(shp, dtype=torch.uint8, device=dev),
             torch.empty(shp, dtype=torch.uint8, device=dev)) for _ in range(slots)]
    d_out = [(torch.empty(shp, dtype=torch.float32, device=dev),
              torch.empty(shp, dtype=torch.float32, device=dev)) for _ in range(slots)]
    h_out = [(torch.empty(shp, dtype=torch.float32).pin_memory(),
              torch.empty(shp, dtype=torch.float32).pin_memory()) for _ in range(slots)]
    ws = [hsflow.alloc_workspace(rows, cols, batch, dev) for _ in range(slots)]
    s_h2d, s_cmp, s_d2h = (torch.cuda.Stream(dev) for _ in range(3))
    ev = {k: [torch.cuda.Event() for _ in range(slots)]
          for k in ("in", "done", "in_free", "out_free")}

    def solve(sl, s):
        hsflow.flow_device(d_in[sl][0], d_in[sl][1], args.window, iters, args.alpha,
                           d_out[sl][0], d_out[sl][1], ws[sl], s)

    # each slot's solve is one hipGraph, as in the resident leg: eager, the
    # ~100 dependent launches of a solve leave dispatch gaps on the GPU
    graphs = [None] * slots
    if not args.no_graph:
        try:
            cur = torch.cuda.current_stream(dev)
            for sl in range(slots):
                cap = torch.cuda.Stream(dev)
                cap.wait_stream(cur)
                with torch.cuda.stream(cap):
                    solve(sl, cap)  # eager once: library side streams exist
                cur.wait_stream(cap)
                torch.cuda.synchronize(dev)
                g = torch.cuda.CUDAGraph()
                with hsflow.max_streams_as(2), \
                        torch.cuda.graph(g, capture_error_mode="thread_local"):
                    solve(sl, torch.cuda.current_stream(dev))
                graphs[sl] = g
            torch.cuda.synchronize(dev)
        except Exception as e:  # pragma: no cover - eager fallback, reported
            print(f"bench: e2e graph capture failed ({e}); eager solves", file=sys.stderr)
            graphs = [None] * slots

    def run(n):
        for k in range(n):
            sl = k % slots
            a, b = host_in[k % 2]
            with torch.cuda.stream(s_h2d):
                if k >= slots:
                    s_h2d.wait_event(ev["in_free"][sl])
                d_in[sl][0].copy_(a, non_blocking=True)
                d_in[sl][1].copy_(b, non_blocking=True)
                ev["in"][sl].record(s_h2d)
            with torch.cuda.stream(s_cmp):
                s_cmp.wait_event(ev["in"][sl])
                if k >= slots:
                    s_cmp.wait_event(ev["out_free"][sl])
                if graphs[sl] is not None:
                    graphs[sl].replay()  # on s_cmp, the current stream
                else:
                    solve(sl, s_cmp)
                ev["in_free"][sl].record(s_cmp)
                ev["done"][sl].record(s_cmp)
            with torch.cuda.stream(s_d2h):
                s_d2h.wait_event(ev["done"][sl])
                hsflow.download_device(h_out[sl][0], d_out[sl][0], s_d2h)
                hsflow.download_device(h_out[sl][1], d_out[sl][1], s_d2h)
                ev["out_free"][sl].record(s_d2h)
        torch.cuda.synchronize(dev)

    # warm-up, untimed, by time like the resident legs' pre-warm: the first
    # pipelined run of a process read 4.6-4.7 ms per batch and every later
    # one 4.15 (scripts/e2e_slots_ab.py, profiles/r04_e2e_slots_ab.jsonl),
    # also after 12 untimed batches; copies and solves together need
    # longer than the solves alone to reach their steady rate
    t_end = time.perf_counter() + E2E_WARM_S
    while True:
        run(slots)
        if time.perf_counter() >= t_end:
            break
    # each stage of a batch alone on this box, after the warm-up (the
    # pipeline's bound is the slowest of them plus their contention): the
    # upload, the solve, the download -- the box-to-box spread of the e2e
    # rate follows these
    def alone(fn, reps=5, warm_s=0.0):
        # the solve gets the resident legs' pre-warm (the clock needs ~0.1 s
        # of load to settle: measured cold, the same graph reads 3.98 ms
        # against 3.6 ms, scripts/e2e_slot_probe.py)
        fn()
        torch.cuda.synchronize(dev)
        t_end = time.perf_counter() + warm_s
        while time.perf_counter() < t_end:
            fn()
            torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / reps * 1e3

    def up():
        with torch.cuda.stream(s_h2d):
            d_in[0][0].copy_(host_in[0][0], non_blocking=True)
            d_in[0][1].copy_(host_in[0][1], non_blocking=True)

    def sv():
        with torch.cuda.stream(s_cmp):
            if graphs[0] is not None:
                graphs[0].replay()
            else:
                solve(0, s_cmp)

    def down():
        hsflow.download_device(h_out[0][0], d_out[0][0], s_d2h)
        hsflow.download_device(h_out[0][1], d_out[0][1], s_d2h)

    stage_ms = {"h2d": round(alone(up), 3), "solve": round(alone(sv, warm_s=0.15), 3),
                "d2h": round(alone(down), 3)}
    t = time.perf_counter()
    run(n_batches)
    dt = time.perf_counter() - t
    # the last batch's flow arrived intact on the host
    last = (n_batches - 1) % slots
    ok = bool(torch.isfinite(h_out[last][0]).all()) and \
        bool(torch.equal(h_out[last][0], d_out[last][0].cpu())) and \
        bool(torch.equal(h_out[last][1], d_out[last][1].cpu()))

    mb_in, mb_out = 2 * batch * rows * cols / 1e6, 2 * batch * rows * cols * 4 / 1e6
    return {"pairs_per_s_e2e": round(n_batches * batch / dt, 2),
            "e2e": {"workload": f"{wl_name}, {batch} pairs per batch, {n_batches} batches "
                                f"({n_batches * batch} pairs)",
                    "input": "pinned host u8 gray frames", "output": "pinned host f32 u, v",
                    "ms_per_batch": round(dt / n_batches * 1e3, 3), "slots": slots,
                    "solve": "hipGraph replay" if graphs[0] is not None else "eager",
                    "stage_ms_alone": stage_ms,
                    "link_gbps": {"h2d": round(mb_in / stage_ms["h2d"], 1),
                                  "d2h": round(mb_out / stage_ms["d2h"], 1)},
                    "finite": ok}}


# --------------------------------------------------------------- stream
def _transport(world, dev):
    """What moved the stream leg's pairs: RCCL only for CUDA tensors under
    the nccl backend (the gloo rehearsal on one GPU stages through the host
    and says so)."""
    if world == 1:
        return "none (one rank)"
    import torch.distributed as dist
    backend = dist.get_backend()
    if backend == "nccl" and dev.type == "cuda":
        return "RCCL point-to-point"
    return f"{backend} ({dev.type} tensors)"


def stream_leg(wl_name, args, world, rank, dev, solve_batch=None, n_pairs=None, ref=None,
               golden=None):
    """BASELINE config 4: a stream of n_pairs synthetic frame pairs held by
    rank 0, scattered one-per-rank round-robin (point-to-point over RCCL;
    gloo in the CPU tests), each rank's share solved in one batched call,
    (u, v) gathered back to rank 0.  Timed end to end, max over ranks.

    Checked on rank 0 after the timed passes: pair 0 (seed 1000) against
    `golden`, and pairs 0..k-1 bit for bit against `ref` = (u, v) of the
    same seeds from the resident leg (frame pairs are independent and K2 is
    bit-identical for any batch, split or blocking depth), so a mis-routed
    or mis-ordered scatter or gather cannot pass."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import frame_parallel as fp
    import hsflow

    wl = WORKLOADS[wl_name]
    rows, cols = wl["rows"], wl["cols"]
    iters = args.iters or wl["iters"]
    n = n_pairs or args.pairs
    stream = None
    if rank == 0:
        # the stream's frames back to back in one device buffer per frame
        # slot (as a decoder writing into one allocation leaves them): a
        # group of consecutive pairs is then a view, not a stacked copy
        # (frame_parallel.batch_of).  8-bit gray frames, the type the
        # reference's frames have after main.cpp:13-14: a quarter of f32's
        # bytes over rank 0's links, and K1 packs the same exact gradients
        # from them as from the f32 frames of the resident leg (the bitwise
        # check against it below)
        A = torch.empty((n, rows, cols), dtype=torch.uint8, device=dev)
        B = torch.empty_like(A)
        for j in range(n):
            a, b = hsflow.synth_pair(1000 + j, rows, cols)
            A[j].copy_(torch.from_numpy(a.astype(np.uint8)))
            B[j].copy_(torch.from_numpy(b.astype(np.uint8)))
        stream = [(A[j], B[j]) for j in range(n)]
    mine = fp.my_pairs(n, rank, world)
    # each rank's share in groups (frame_parallel.group_sizes, the same on
    # every rank): one rank, batches of at most 8 pairs (8 pairs fill the
    # chip, and a group's planes, ~330 MB per pass, partly stay in the 256 MB
    # Infinity Cache between passes, which 64 pairs in one call do not: one
    # rank solved 64 pairs at 1.27 M Mpix*iter/s in one call against 1.35 M
    # for 8-pair batches); N > 1, the sizes that minimise the pipeline model
    # (a large first group solves while the next ones arrive, small last
    # groups keep the exposed return of the last (u, v) short;
    # frame_parallel.run_stream_pipelined, scripts/scale_predict.py)
    in_mb, out_mb = 2 * rows * cols / 1e6, 2 * rows * cols * 4 / 1e6
    # the model's link rate measured on this node's links before the timed
    # passes (one f32 plane per round trip, rank 0 to each peer; the slowest
    # peer's rate, broadcast so every rank picks the same groups), in place
    # of the assumed frame_parallel.LINK_GBPS
    link = fp.measure_link_gbps(dev, rank, world, rows * cols * 4) if world > 1 else None
    link_gbps = link["link_gbps"] if link else fp.LINK_GBPS

    def sizes(share):
        return fp.group_sizes(share, world, in_mb, out_mb, link_gbps=link_gbps)

    my_sizes = sizes(len(mine))
    if solve_batch is None:
        ws = hsflow.alloc_workspace(rows, cols, max(my_sizes), dev)

        def solve_batch(I0, I1):
            return hsflow.flow_device(I0, I1, args.window, iters, args.alpha, workspace=ws)

    out = [None]

    def one_pass():
        out[0] = fp.run_stream_pipelined(stream, n, (rows, cols), torch.uint8, solve_batch,
                                         dev, rank, world, sizes=sizes)

    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    warm = None
    if dev.type == "cuda":
        # untimed, rank-local clock warm-up: the rank's solve of one group of
        # its own size, no collective inside, so ranks may run different
        # counts (prewarm's rule); the timed passes are unchanged
        g = max(my_sizes)
        gen = torch.Generator(device=dev).manual_seed(rank)
        W0, W1 = (torch.rand((g, rows, cols), generator=gen, device=dev) * 255 for _ in "01")
        n_w, t_w = prewarm(lambda: solve_batch(W0, W1), sync)
        warm = {"prewarm_steps": n_w, "prewarm_s": round(t_w, 3), "pairs": g}
        del W0, W1
    if world > 1:
        dist.barrier()  # every rank's communicator is up before the first P2P call
    steps = max(1, min(args.steps, 3))
    elapsed = timed_region(one_pass, sync, steps, 1, world, dev)
    leg = {"pairs_per_s": round(n * steps / elapsed, 2),
           "ms_per_pass": round(elapsed / steps * 1e3, 3), "pairs": n,
           "groups_per_rank": len(my_sizes), "group_sizes": my_sizes,
           "link_gbps_measured": (round(link["measured_gbps"], 3) if link else None),
           "link_gbps_per_peer": (link["per_peer"] if link and rank == 0 else None),
           "link_gbps_model": round(link_gbps, 2),
           "frames": "u8",
           "Mpix_iter_per_s": round(n * steps * rows * cols * iters / elapsed / 1e6, 1),
           "transport": _transport(world, dev),
           "scaling": "strong"}
    if warm is not None:
        leg["untimed_prewarm"] = warm
    if rank == 0:
        res = out[0]
        leg["gathered"] = len(res) if res is not None else 0
        leg["finite"] = bool(res is not None and all(bool(torch.isfinite(u).all())
                                                      for u, _ in res[:2]))
        par = {"ok": bool(leg["finite"] and leg["gathered"] == n)}
        if golden is not None and res:
            g = parity_check(res[0][0].cpu().numpy(), res[0][1].cpu().numpy(), golden)
            par["pair0"] = g
            par["ok"] = par["ok"] and bool(g["ok"])
        if ref is not None and res:
            k = min(len(ref[0]), len(res))
            same = [bool(torch.equal(res[j][0], ref[0][j]) and torch.equal(res[j][1], ref[1][j]))
                    for j in range(k)]
            par["bitwise_vs_resident"] = {"pairs": k, "identical": sum(same)}
            par["ok"] = par["ok"] and all(same)
        leg["parity"] = par
    return leg


# --------------------------------------------------------------- main
def main():
    args = parse()
    bad = refuse_diagnostics()
    if bad:
        print(f"bench: refusing to run with diagnostic variables set: {bad}", file=sys.stderr)
        sys.exit(2)
    action, world = world_from_env(args.gpus)
    if action == "refuse":
        print(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks; "
              "refusing to report a line for the wrong GPU count", file=sys.stderr)
        sys.exit(2)
    if action == "launch":
        sys.exit(launch_ranks(world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:
        sys.exit(launch_check(world, rank))

    import torch
    import torch.distributed as dist
    import hsflow

    if hsflow.is_probe_build():  # hsflow_build_flags() != 0: not the product build
        print(f"bench: {hsflow.LIB_PATH} was built with development flags; rebuild the "
              "product library", file=sys.stderr)
        sys.exit(2)
    # HSFLOW_BENCH_BACKEND=gloo + HSFLOW_BENCH_DEVICE=0: rehearse the N > 1
    # logic with several ranks on one GPU (diagnostics; the driver's runs
    # use RCCL, one GPU per rank)
    backend = os.environ.get("HSFLOW_BENCH_BACKEND", "nccl")
    dev = torch.device("cuda", int(os.environ.get("HSFLOW_BENCH_DEVICE", local)))
    torch.cuda.set_device(dev)

    state = {"up": False}

    def init_dist():
        if world > 1 and not state["up"]:
            # a collective that never completes (a mismatched RCCL
            # send/recv order, a dead peer) aborts the run after 5 minutes
            # instead of holding the node; every leg takes well under that
            import datetime
            limit = datetime.timedelta(minutes=5)
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=dev, timeout=limit)
            else:
                dist.init_process_group(backend, timeout=limit)
            state["up"] = True

    if args.mode == "stream":
        init_dist()
        golden = golden_entry(WORKLOADS[args.workload]["rows"], WORKLOADS[args.workload]["cols"],
                              args.iters or WORKLOADS[args.workload]["iters"], args.window, 1,
                              args.alpha) if rank == 0 else None
        leg = stream_leg(args.workload, args, world, rank, dev, golden=golden)
        status = 0
        if rank == 0:
            print(json.dumps({
                "metric": "frame-pairs/s (config 4 stream: RCCL scatter + solve + gather)",
                "value": leg["pairs_per_s"], "unit": "pairs/s", "n_gpus": world,
                "steps": max(1, min(args.steps, 3)), "warmup": 1,
                "ms_per_step": leg["ms_per_pass"], "higher_is_better": True,
                "scaling": "strong", "vs_baseline": None, "dtype": "f32",
                "data": "synthetic f32 frame pairs",
                "config": {"workload": f"stream of {leg['pairs']} x {args.workload} pairs",
                           "parallelism": f"frame-parallel x{world}"},
                "stream": leg}), flush=True)
            status = 0 if leg["parity"]["ok"] else 3
        if world > 1:
            dist.destroy_process_group()
        sys.exit(status)
    if args.mode == "bands":
        init_dist()
        return bands_mode(args, world, rank, dev)

    default_run = (args.workload == "1080p" and not args.iters and not args.batch and
                   args.window == 5 and args.alpha == 1.0 and not args.levels and
                   not args.dtype)
    if args.kb:
        hsflow.set_iters_per_launch(args.kb)
    keep = default_run and not args.no_stream
    progress(f"resident {args.workload}", rank)
    prim = resident_leg(args.workload, args, dev, world, rank, init_dist, keep=keep)
    resident_ref = None
    if keep:
        prim, resident_ref = prim
    sec = c5 = w3 = None
    singles = {}
    if default_run and not args.no_secondary:
        progress("resident 4k", rank)
        sec = resident_leg("4k", args, dev, world, rank)
    if default_run and not args.no_w3:
        # windowSize 5 is the headline, report 3 (north_star) too
        progress("resident 1080p w3", rank)
        w3 = resident_leg("1080p", args, dev, world, rank, window=3)
    if default_run and not args.no_8k:
        progress("resident 8k pyramid", rank)
        c5 = resident_leg("8k", args, dev, world, rank)
    if default_run and not args.no_single:
        # configs[1] / configs[2] as stated: one pair per solve (main.cpp:97-98)
        for wl in ("1080p", "4k"):
            progress(f"single pair {wl}", rank)
            singles[wl] = resident_leg(wl, args, dev, world, rank, batch=1)
    stream_peak = hbm_stream_peak(dev) if rank == 0 else None
    e2e = None
    if not args.no_e2e and args.workload != "8k" and rank == 0:
        e2e = e2e_leg(args.workload, args, dev)
    strm = None
    if default_run and not args.no_stream:
        golden = golden_entry(1080, 1920, 300, 5, 1, 1.0) if rank == 0 else None
        progress("stream (configs[3])", rank)
        strm = stream_leg("1080p", args, world, rank, dev, ref=resident_ref, golden=golden)
    del resident_ref
    bands = None
    if default_run and not args.no_bands:
        # BASELINE configs[4] as stated for N GPUs: one 8K pair in N row
        # bands, halo rows over RCCL (at N = 1: one band, no exchange)
        init_dist()
        progress("bands (configs[4])", rank)
        bands = bands_leg(args, world, rank, dev, steps=max(1, min(args.steps, 5)), warmup=1)

    if default_run and rank == 0:
        progress("config1 + host_api", rank)
    c1 = config1_leg(dev) if (default_run and rank == 0) else None
    host_api = host_api_leg() if (default_run and rank == 0 and not args.no_host_api) else None
    cpu = cpu_all = None
    if rank == 0 and not args.no_cpu_baseline:
        progress("cpu baseline", rank)
        # on every line, N > 1 included: the host-core figure the GPU counts
        # are read against (north_star)
        cpu = cpu_baseline(prim["rows"], prim["cols"], args.window, args.alpha,
                           args.cpu_iters)
        # SURVEY §8(d) second CPU line: all cores of the box's CPU share
        # (16 per GPU on the MI355X pool; os.cpu_count() shows the machine)
        n_thr = min(16, os.cpu_count() or 1)
        cpu_all = cpu_baseline(prim["rows"], prim["cols"], args.window, args.alpha,
                               args.cpu_iters, n_thr)
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        if sec is not None:
            # the CPU line per config -- 4K on 1 thread, bounded
            sec["cpu_baseline"] = cpu_baseline(sec["rows"], sec["cols"], args.window,
                                               args.alpha, args.cpu_iters or 20)
        if c5 is not None:
            # the 8K level-0 plane, 1 thread, 4 iterations (~6 s)
            c5["cpu_baseline"] = cpu_baseline(c5["rows"], c5["cols"], args.window,
                                              args.alpha, args.cpu_iters or 4)

    status = 0
    if rank == 0:
        line = {
            "metric": "Mpix*iter/s (Horn-Schunck Jacobi) + frame-pairs/s",
            "value": prim["value"],
            "unit": "Mpix*iter/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": prim["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic {prim['input_dtype']} frame pairs (hash texture, shift "
                    "(-0.75,+1.5) px)",
            "config": {k: prim[k] for k in ("workload", "rows", "cols", "iters", "window",
                                            "levels", "input_dtype", "alpha",
                                            "pairs_per_gpu_per_step", "step")},
            "pairs_per_s_resident": prim["pairs_per_s_resident"],
            "untimed_prewarm": prim["untimed_prewarm"],
            "parity": prim["parity"],
            "roofline": prim["roofline"],
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_all,
        }
        line["config"]["parallelism"] = f"frame-parallel x{world}"
        line["config"]["iters_per_launch"] = prim["roofline"]["iters_per_launch"]
        line["config"]["kernel"] = prim["roofline"]["kernel"]
        if e2e is not None:
            line.update(e2e)
        keys = ("workload", "value", "unit", "ms_per_step", "pairs_per_s_resident", "roofline",
                "parity", "cpu_baseline")
        if sec is not None:
            line["secondary"] = {k: sec[k] for k in keys if k in sec}
        if c5 is not None:
            line["config5"] = {k: c5[k] for k in keys if k in c5}
        if singles:
            line["single_pair"] = {wl: {k: s[k] for k in keys if k in s}
                                   for wl, s in singles.items()}
        if c1 is not None:
            line["config1"] = c1
        if w3 is not None:
            line["window3"] = {k: w3[k] for k in keys if k in w3}
        if stream_peak is not None:
            line["torch_copy_gbps"] = stream_peak
        if strm is not None:
            line["stream"] = strm
        if bands is not None:
            line["bands"] = bands
        if host_api is not None:
            line["host_api"] = host_api
        # one verdict per BASELINE config
        ha = host_api or {}
        legs = {"configs[0]": [c1], "configs[1]": [prim, singles.get("1080p"), w3,
                                                    ha.get("1080p")],
                "configs[2]": [sec, singles.get("4k"), ha.get("4k")], "configs[3]": [strm],
                "configs[4]": [c5, bands]}
        verdict = {}
        for name, ls in legs.items():
            ps = [l["parity"] for l in ls if l is not None and l.get("parity") is not None]
            oks = [p["ok"] for p in ps if p.get("ok") is not None]
            verdict[name] = (all(oks) if oks else None)
        line["parity_all"] = {"ok": all(v is not False for v in verdict.values()),
                              "configs": verdict}
        print(json.dumps(line), flush=True)
        for leg in (prim, sec, w3, c5, c1, strm, bands, *singles.values(), *ha.values()):
            if leg is not None and leg.get("parity") is not None and \
                    leg["parity"].get("ok") is False:
                print(f"bench: PARITY FAILURE on {leg.get('workload', 'stream')}: "
                      f"{leg['parity']}", file=sys.stderr)
                status = 3
    if world > 1:
        dist.destroy_process_group()
    if status:
        sys.exit(status)


def bands_leg(args, world, rank, dev, steps, warmup, chunk=None, overlap=None, ops=None,
              result=None):
    """BASELINE config 5 across ranks: one pair (the 8k workload, fp16, 3
    levels, 1000 it/level unless the flags say otherwise) split into row
    bands; every `chunk` iterations each rank exchanges halo rows with its
    neighbours (RCCL point-to-point under the nccl backend), and rank 0
    gathers (u, v).  Timed: pyramid build + banded levels + exchanges +
    gather (inputs broadcast from rank 0 beforehand, resident in HBM).
    Strong scaling: the work is fixed.  Rank 0's dict carries the parity of
    the gathered (u, v) against the 8k_w5_l3 golden (bit-identical to the
    single-GPU solve by construction, row_bands.py).  `ops` replaces the
    libhsflow band operations (tests/test_bench_ranks.py runs this leg over
    gloo with the CPU oracle as the band solver); a `result` list receives
    rank 0's gathered (u, v)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import hsflow
    import row_bands as rb
    import blocks as bl

    wl = dict(WORKLOADS[args.workload if args.workload != "1080p" else "8k"])
    rows, cols = wl["rows"], wl["cols"]
    iters = args.iters or wl["iters"]
    levels = args.levels or wl.get("levels", 1)
    in_dtype = args.dtype or wl.get("dtype", "f32")
    window, alpha = args.window, args.alpha
    want_overlap = bool(args.overlap if overlap is None else overlap) and world > 1
    # row bands or a grid of blocks (the overlapped schedule exists for bands)
    split = getattr(args, "split", "auto") or "auto"
    if split == "auto":
        split = "rows" if (want_overlap or world == 1) else "blocks"
    if split == "blocks" and want_overlap:
        print("bench: bands --overlap runs row bands only; blocks without overlap",
              file=sys.stderr)
        want_overlap = False
    # one rank exchanges nothing: its band is the whole plane, solved in one
    # call per level
    if chunk is None:
        spec = args.chunk or (BLOCKS_CHUNK if split == "blocks" else ROWS_CHUNK)
        chunk = ([int(x) for x in str(spec).split(",")] if world > 1 else iters)
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
    # the chunks asked for where their halos fit the bands, shorter where not
    # (e.g. --chunk 24,48 at 8 ranks with window 7); said on stderr
    # coarse levels of at most BANDS_WHOLE_MAX_PX solved whole on every rank:
    # no chunks, no exchanges (row_bands.whole_levels)
    whole = rb.whole_levels(rows, cols, levels, world, BANDS_WHOLE_MAX_PX)
    if split == "blocks":
        p, notes = bl.fit_plan2d(rows, cols, levels, world, window, chunk, whole=whole)
    else:
        p, notes = rb.fit_plan(rows, cols, levels, world, window, chunk, overlap=want_overlap,
                               whole=whole)
    for msg in notes:
        print(f"bench: bands {msg}", file=sys.stderr)
    ops = [ops if ops is not None else rb.DeviceOps(window, alpha, dev)]
    res = [None]

    if split == "blocks":
        comm = bl.DistComm2D() if world > 1 else bl.LocalComm2D()
        overlap = False

        def one():
            states = bl.solve([I0], [I1], p, iters, ops, comm, [rank])
            res[0] = bl.gather_owned(states, p, comm)
    else:
        comm = rb.DistComm() if world > 1 else rb.LocalComm()
        overlap = want_overlap and rb.overlap_ok(p)
        if want_overlap and not overlap:
            print("bench: bands --overlap cannot be used with this plan; plain schedule",
                  file=sys.stderr)
        solve = rb.solve_overlapped if overlap else rb.solve

        def one():
            states = solve([I0], [I1], p, iters, ops, comm, [rank])
            res[0] = rb.gather_owned(states, p, comm)

    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    elapsed = timed_region(one, sync, steps, warmup, world, dev)
    px_all = sum(r * c for r, c in p.sizes)
    exchanges = sum(-(-iters // c) for c, w in zip(p.chunks, p.whole) if not w) \
        if world > 1 else 0
    shape = (f"a {p.grid[0]} x {p.grid[1]} grid of blocks" if split == "blocks" else
             f"{world} row band" + ("s" if world > 1 else ""))
    leg = {"workload": f"{cols}x{rows} {in_dtype}, {levels} levels, {iters} it/level, "
                       f"ws {window}, one pair in {shape}",
           "split": split + (f" {p.grid[0]}x{p.grid[1]}" if split == "blocks" else ""),
           "value": round(px_all * iters * steps / elapsed / 1e6, 1), "unit": "Mpix*iter/s",
           "ms_per_pair": round(elapsed / steps * 1e3, 3), "steps": steps,
           "pairs_per_s": round(steps / elapsed, 2),
           "n_ranks": world, "chunks_per_level": list(p.chunks),
           "whole_levels": [l for l, w in enumerate(p.whole) if w],
           "halo_rows_per_level": list(p.halos),
           "exchanges_per_solve": exchanges,
           "exchange": "overlapped with interior iterations" if overlap else "after every chunk",
           "transport": _transport(world, dev), "scaling": "strong"}
    if rank == 0:
        u, v = (np.asarray(x.cpu().numpy() if hasattr(x, "cpu") else x) for x in res[0])
        golden = golden_entry(rows, cols, iters, window, levels, alpha)
        leg["parity"] = parity_check(u, v, golden)
        if result is not None:
            result.append((u, v))
    del I0, I1, res
    if dev.type == "cuda":
        torch.cuda.empty_cache()
    return leg


def bands_mode(args, world, rank, dev):
    """--mode bands: the bands leg alone, its own JSON line."""
    import torch.distributed as dist
    leg = bands_leg(args, world, rank, dev, args.steps, args.warmup)
    status = 0
    if rank == 0:
        print(json.dumps({
            "metric": "Mpix*iter/s (config 5: one pair split over ranks, halo exchange over RCCL)",
            "value": leg["value"], "unit": "Mpix*iter/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": leg["ms_per_pair"],
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic frame pair",
            "config": {"workload": leg["workload"], "window": args.window,
                       "chunks_per_level": leg["chunks_per_level"],
                       "halo_rows_per_level": leg["halo_rows_per_level"],
                       "exchange": leg["exchange"],
                       "parallelism": f"{leg['split']} x{world}"},
            "parity": leg["parity"], "bands": leg}), flush=True)
        status = 3 if leg["parity"].get("ok") is False else 0
    if world > 1:
        dist.destroy_process_group()
    if status:
        sys.exit(status)


def host_api_leg(reps=15):
    """The reference's own call as a drop-in sees it (main.cpp:97-98;
    hornSchunck.cpp:43-75): ONE pair of pageable host u8 gray frames through
    hsflow_flow (upload, K1, the Jacobi passes, download) to float64
    (CV_64FC1) u, v, blocking.  Outputs reused across calls as
    cv::Mat::create() keeps them (the adapter's steady state in a frame
    loop); the first-touch cost of fresh output pages is reported beside it,
    as is f32 output.  Median of `reps`; parity of the f64 output against
    the committed golden (u, v) of seed 1000."""
    import numpy as np
    import hsflow
    out = {}
    for wl in ("1080p", "4k"):
        w = WORKLOADS[wl]
        rows, cols, iters = w["rows"], w["cols"], w["iters"]
        I0, I1 = hsflow.synth_pair(1000, rows, cols, dtype=np.uint8)
        hs = hsflow.hornSchunck(5, iters, 1.0)
        u = np.empty((rows, cols), np.float64)
        v = np.empty((rows, cols), np.float64)
        hs.getFlow(I0, I1, u, v)  # warm: contexts, buffers, pool threads

        def med(fn, n=reps):
            ts = []
            for _ in range(n):
                t = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t)
            return sorted(ts)[len(ts) // 2] * 1e3

        u.fill(np.nan)
        v.fill(np.nan)
        ms = med(lambda: hs.getFlow(I0, I1, u, v))
        par = parity_check(u, v, golden_entry(rows, cols, iters, 5, 1, 1.0))
        # fresh outputs as main.cpp:93 has them (`cv::Mat u, v;` per call):
        # new anonymous pages every call, mapped outside the timed call
        # (np.empty would reuse glibc's freed chunks below its mmap
        # threshold, i.e. pages already faulted in)
        ts = []
        for _ in range(max(3, reps * 3 // 5)):
            # private anonymous pages, as malloc gives a cv::Mat (mmap.mmap's
            # default MAP_SHARED would be shmem, which faults differently)
            m = mmap.mmap(-1, 2 * rows * cols * 8,
                          flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
            fu, fv = np.frombuffer(m, np.float64).reshape(2, rows, cols)
            t = time.perf_counter()
            hs.getFlow(I0, I1, fu, fv)
            ts.append(time.perf_counter() - t)
            fu_ok = bool(np.array_equal(fu, u) and np.array_equal(fv, v))
            del fu, fv
            m.close()
            if not fu_ok:
                par = dict(par, ok=False, fresh_outputs_differ=True)
        ms_fresh = sorted(ts)[len(ts) // 2] * 1e3
        ctx = hs._c()
        u32 = np.empty((rows, cols), np.float32)
        v32 = np.empty((rows, cols), np.float32)
        ms_f32 = med(lambda: ctx.flow(I0, I1, 5, iters, 1.0, out_dtype=np.float32,
                                      out=(u32, v32)), max(3, reps // 3))
        out[wl] = {"workload": f"{cols}x{rows} u8 pair, ws 5, alpha 1, {iters} it",
                   "ms_per_call": round(ms, 3),
                   "Mpix_iter_per_s": round(rows * cols * iters / ms / 1e3, 1),
                   "output": "CV_64FC1 (float64), buffers reused (cv::Mat::create)",
                   "ms_per_call_fresh_outputs": round(ms_fresh, 3),
                   "fresh_outputs": "new private anonymous pages per call (mmap)",
                   "ms_per_call_f32_outputs": round(ms_f32, 3),
                   "parity": par}
    return out


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
