"""Predicted N = 1/2/4/8 values of the two multi-GPU legs of bench.py, built
from pieces measured on ONE GPU plus two stated link constants (the 8-GPU
runs are the driver's; DESIGN.md §6 "Predictions" quotes this output).

    python scripts/scale_predict.py > profiles/r04_scale_prediction.json

stream leg (configs[3]): 64 1080p pairs held by rank 0 as u8 frames; rank r
  solves pairs r, r + N, ...; rank 0 sends 2 x 2.07 MB of frames per pair to
  its owner and receives 2 x 8.3 MB of (u, v) back.  A rank's share goes in
  the groups frame_parallel.group_sizes picks (bench.stream_leg).
  Measured: the resident solve time of batches of 1..8 pairs.  Modelled
  (frame_parallel.pipeline_ms): rank 0 sends a group to every rank at once,
  each link at LINK_GBPS (RCCL point-to-point over xGMI); group c+1 travels
  while group c is solved, group c's (u, v) return while later groups are
  solved, the last group's return is exposed.
bands leg (configs[4] as stated for N GPUs): one 8K fp16 pair, 3 levels x
  1000 it, rank r solves its extended band in chunks (24 iterations at level
  0, 48 at the coarser levels: bench.py's default) with a halo exchange
  after each.  Measured: per level, the GPU time and
  the host issue time of one chunk on the largest extended band (eager
  jacobi_device calls, as row_bands.solve issues them), K1 per level, the
  pyramid build.  Modelled: an exchange costs XCHG_US of latency plus its
  transfer on the critical path (2 x 2 RCCL sends and receives of H rows of
  u and v each, H x cols x 8 bytes per neighbour at LINK_GBPS, the two
  neighbours on separate links) and the host issues an exchange in
  XCHG_HOST_US; per chunk the slower of the GPU (chunk + exchange) and the
  host (issue) sets the pace; the final gather moves the owned rows of
  (u, v) to rank 0 at LINK_GBPS.
  The overlapped schedule (row_bands.solve_overlapped): the middle rank's
  chunk loop is timed on the GPU with the transfers left out (NullComm),
  which gives max(host, interior || strips) per chunk; the exchange then
  only has to land before the strips start: per chunk the slower of that
  loop (+ XCHG_HOST_US of posting) and XCHG_US + transfer + the strips'
  GPU time.  The leg runs the cheaper schedule the plan allows."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cpp-optical-flow_amd"), ROOT]
import blocks as bl  # noqa: E402
import frame_parallel as fp  # noqa: E402
import hsflow  # noqa: E402
import row_bands as rb  # noqa: E402

LINK_GBPS = fp.LINK_GBPS  # RCCL p2p per peer over one xGMI link (~1/3 of the 153 GB/s raw)
XCHG_US = 40.0       # one halo exchange on the critical path (RCCL p2p latency)
XCHG_HOST_US = 120.0  # host time to post one exchange (clones + batch_isend_irecv)


def resident_ms(batch, reps=6):
    rows, cols, iters = 1080, 1920, 300
    ps = [hsflow.synth_pair(1000 + i, rows, cols) for i in range(batch)]
    I0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
    I1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
    u = torch.empty((batch, rows, cols), dtype=torch.float32, device="cuda")
    v = torch.empty_like(u)
    ws = hsflow.alloc_workspace(rows, cols, batch)
    hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws)
    t_end = time.perf_counter() + 0.15
    while time.perf_counter() < t_end:
        hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def group_solve_ms(reps=6):
    """Resident solve time of a batch of g 1080p pairs, g = 1..8 (the table
    frame_parallel.GROUP_SOLVE_MS restates)."""
    return [round(resident_ms(g, reps), 4) for g in range(1, 9)]


def stream_prediction(n, solve_ms, pairs=64, link_gbps=None):
    """The stream leg at N ranks: rank 0 keeps pairs 0, N, 2N, ... and sends
    every other pair's two u8 frames to its owner; each rank's share goes in
    frame_parallel.group_sizes groups (the bench's rule, with the measured
    batch solve times); frame_parallel.pipeline_ms models a remote rank's
    pass (its groups' frames arriving over its link from rank 0, solves,
    (u, v) back over the other direction), rank 0's own share has no
    transfers.  The slowest rank sets the pass."""
    link = LINK_GBPS if link_gbps is None else link_gbps
    per = pairs // n
    in_mb = 2 * 1080 * 1920 / 1e6        # two u8 frames
    out_mb = 2 * 1080 * 1920 * 4 / 1e6   # u, v in f32
    sizes = fp.group_sizes(per, n, in_mb, out_mb, solve_ms, link)
    own = fp.group_sizes(per, 1, in_mb, out_mb, solve_ms, link)
    t0 = fp.pipeline_ms(own, in_mb, out_mb, solve_ms, link, remote=False)
    t0 = fp.pipeline_ms(sizes, in_mb, out_mb, solve_ms, link, remote=False) \
        if n > 1 else t0
    tr = fp.pipeline_ms(sizes, in_mb, out_mb, solve_ms, link) if n > 1 else 0.0
    total = max(t0, tr)
    return {"n": n, "link_gbps": link, "pairs_per_rank": per, "group_sizes": sizes,
            "rank0_ms": round(t0, 3), "remote_rank_ms": round(tr, 3),
            "frames": "u8", "ms_per_pass": round(total, 3),
            "pairs_per_s": round(pairs / total * 1e3, 1)}


def chunk_costs(rows, cols, chunk, nchunks=12, batch=1):
    """GPU ms and host ms of one eager chunk on a rows x cols band (a stack
    of `batch` such planes)."""
    ps = [hsflow.synth_pair(1000 + i, rows, cols) for i in range(batch)]
    t0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda().half()
    t1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda().half()
    ws = hsflow.alloc_workspace(rows, cols, batch)
    u = torch.zeros((batch, rows, cols), dtype=torch.float32, device="cuda")
    v = torch.zeros_like(u)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    k1 = time.perf_counter()
    hsflow.gradients_device(t0, t1, ws)
    torch.cuda.synchronize()
    k1 = (time.perf_counter() - k1) * 1e3
    for _ in range(3):
        hsflow.jacobi_device(rows, cols, batch, 5, chunk, 1.0, u, v, ws, warm_start=True)
    torch.cuda.synchronize()
    host = []
    e0.record()
    for _ in range(nchunks):
        h = time.perf_counter()
        hsflow.jacobi_device(rows, cols, batch, 5, chunk, 1.0, u, v, ws, warm_start=True)
        host.append((time.perf_counter() - h) * 1e3)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / nchunks, float(np.median(host)), k1


class NullComm:
    """The exchanges of one rank with the transfers left out: the rank's
    chunk loop alone (its host issue and its GPU work), for timing."""

    def start(self, states, level):
        return None

    def wait(self, handle):
        pass

    def exchange(self, states, level):
        pass

    def start_strips(self, states):
        return None


def loop_chunk_ms(n, R, C, chunk, overlapped, short=2, long=10, reps=3):
    """Wall ms per chunk of the middle rank's chunk loop on one level of
    R x C in N bands (row_bands.solve or solve_overlapped, NullComm): the
    difference of a long and a short run, so the level's set-up drops out."""
    p = rb.plan(R, C, 1, n, 5, chunk)
    if overlapped and not rb.overlap_ok(p):
        return None
    a, b = hsflow.synth_pair(1000, R, C)
    I0 = torch.from_numpy(a).cuda().half()
    I1 = torch.from_numpy(b).cuda().half()
    solver = rb.solve_overlapped if overlapped else rb.solve
    rank = n // 2

    def run(k):
        ops = rb.DeviceOps(5, 1.0, torch.device("cuda"))
        torch.cuda.synchronize()
        t = time.perf_counter()
        solver([I0], [I1], p, k * chunk, [ops], NullComm(), [rank])
        torch.cuda.synchronize()
        return time.perf_counter() - t

    run(short)
    ts = float(np.median([run(short) for _ in range(reps)]))
    tl = float(np.median([run(long) for _ in range(reps)]))
    return max(tl - ts, 0.0) / (long - short) * 1e3


def _level_plain(n, ext, C, ck, H, iters):
    g, h, k1 = chunk_costs(ext, C, ck)
    nch = -(-iters // ck)
    xfer = H * C * 8 / 1e6 / LINK_GBPS if n > 1 else 0.0  # ms per exchange
    per = max(g + (XCHG_US / 1e3 + xfer if n > 1 else 0.0),
              h + (XCHG_HOST_US / 1e3 if n > 1 else 0.0))
    return nch * per + k1, {"band_rows": ext, "cols": C, "chunks": nch, "chunk": ck,
                            "halo_rows": H, "gpu_ms_per_chunk": round(g, 4),
                            "host_ms_per_chunk": round(h, 4),
                            "exchange_transfer_ms": round(xfer, 4),
                            "ms_per_chunk": round(per, 4)}


def _level_overlapped(n, R, C, ck, H, iters, k1):
    loop = loop_chunk_ms(n, R, C, ck, True)
    sg, _, _ = chunk_costs(3 * H, C, ck, batch=2)
    xfer = H * C * 8 / 1e6 / LINK_GBPS
    per = max(loop + XCHG_HOST_US / 1e3, XCHG_US / 1e3 + xfer + sg)
    nch = -(-iters // ck)
    return nch * per + k1, {"cols": C, "chunks": nch, "chunk": ck, "halo_rows": H,
                            "loop_ms_per_chunk": round(loop, 4),
                            "strips_gpu_ms_per_chunk": round(sg, 4),
                            "exchange_transfer_ms": round(xfer, 4),
                            "ms_per_chunk": round(per, 4)}


def bands_prediction(n, chunk=(24, 48), iters=1000, whole_px=2_200_000, overlap=True):
    """bench.py's plans (row_bands.fit_plan; coarse levels of <= whole_px
    pixels solved whole on every rank, no exchanges): the plain schedule,
    and the overlapped one where its plan allows it; the leg runs the
    cheaper."""
    whole = rb.whole_levels(4320, 7680, 3, n, whole_px)
    out = {"n": n}
    totals = {}
    own = 4320 // n * 7680 * 8 / 1e6  # MB of (u, v) per remote rank
    gather = own / LINK_GBPS if n > 1 else 0.0
    out["gather_ms"] = round(gather, 3)
    k1s = {}
    for sched in ("plain", "overlapped"):
        if sched == "overlapped" and (not overlap or n == 1):
            continue
        p, notes = rb.fit_plan(4320, 7680, 3, n, 5, chunk if n > 1 else iters,
                               overlap=sched == "overlapped", whole=whole)
        if sched == "overlapped" and not rb.overlap_ok(p):
            continue
        rec = {"chunks_per_level": list(p.chunks), "halo_rows_per_level": list(p.halos),
               "notes": notes, "levels": []}
        total = gather
        for l in range(p.levels - 1, -1, -1):
            R, C = p.sizes[l]
            ext = max(b.e1 - b.e0 for b in p.bands[l])
            if p.whole[l]:  # the whole plane in one call, no exchange
                g, h, k1 = chunk_costs(ext, C, iters, nchunks=3)
                lvl = max(g, h) + k1
                rec["levels"].append({"level": l, "band_rows": ext, "cols": C, "whole": True,
                                      "gpu_ms": round(g, 4), "ms": round(lvl, 3)})
            elif sched == "plain":
                lvl, d = _level_plain(n, ext, C, p.chunks[l], p.halos[l], iters)
                k1s[l] = lvl - d["chunks"] * d["ms_per_chunk"]
                rec["levels"].append(dict(level=l, ms=round(lvl, 3), **d))
            else:
                lvl, d = _level_overlapped(n, R, C, p.chunks[l], p.halos[l], iters,
                                           k1s.get(l, 0.0))
                rec["levels"].append(dict(level=l, ms=round(lvl, 3), **d))
            total += lvl
        rec["ms_per_pair"] = round(total, 2)
        out[sched] = rec
        totals[sched] = total
    best = min(totals, key=totals.get)
    out["schedule"] = best
    out["ms_per_pair"] = round(totals[best], 2)
    return out


def blocks_prediction(n, chunk=(24, 48), iters=1000, whole_px=2_200_000):
    """The 2-D block split (blocks.py, bench.py --split blocks): per level
    the largest extended block solved in chunks (GPU time measured on a
    dense plane of that shape), each exchange XCHG_US of latency plus its
    largest message (every peer on a link of its own: edges of H rows or
    columns of u and v, corners) at LINK_GBPS, its host posting
    XCHG_HOST_US per two peers (the bands' constant is for two); per chunk
    the slower of the GPU and the host sets the pace.  Coarse levels of at
    most whole_px pixels solved whole on every rank, as for the bands; the
    gather moves the owned blocks (u, v) to rank 0 at LINK_GBPS."""
    whole = rb.whole_levels(4320, 7680, 3, n, whole_px)
    p, notes = bl.fit_plan2d(4320, 7680, 3, n, 5, chunk if n > 1 else iters, whole=whole)
    own = max((b.b - b.a) * (b.d - b.c) for b in p.blocks[0]) * 8 / 1e6
    gather = own / LINK_GBPS if n > 1 else 0.0
    rec = {"n": n, "grid": list(p.grid), "chunks_per_level": list(p.chunks),
           "halo_per_level": list(p.halos), "notes": notes, "gather_ms": round(gather, 3),
           "levels": []}
    total = gather
    for l in range(p.levels - 1, -1, -1):
        big = max(p.blocks[l], key=lambda b: (b.e1 - b.e0) * (b.f1 - b.f0))
        R, C = big.shape()
        if p.whole[l] or n == 1:
            g, h, k1 = chunk_costs(R, C, iters, nchunks=3)
            lvl = max(g, h) + k1
            rec["levels"].append({"level": l, "block": [R, C], "whole": True,
                                  "gpu_ms": round(g, 4), "ms": round(lvl, 3)})
            total += lvl
            continue
        ck, H = p.chunks[l], p.halos[l]
        g, h, k1 = chunk_costs(R, C, ck)
        nch = -(-iters // ck)
        peers = max(len(bl.halo_sources(p, l, r)) for r in range(n))
        msg = max(max(H * (b.d - b.c), H * (b.b - b.a)) for b in p.blocks[l]) * 8 / 1e6
        xfer = msg / LINK_GBPS
        per = max(g + XCHG_US / 1e3 + xfer, h + XCHG_HOST_US / 1e3 * peers / 2)
        lvl = nch * per + k1
        rec["levels"].append({"level": l, "block": [R, C], "chunks": nch, "chunk": ck,
                              "halo": H, "peers": peers, "gpu_ms_per_chunk": round(g, 4),
                              "host_ms_per_chunk": round(h, 4),
                              "exchange_transfer_ms": round(xfer, 4),
                              "ms_per_chunk": round(per, 4), "ms": round(lvl, 3)})
        total += lvl
    rec["ms_per_pair"] = round(total, 2)
    return rec


def main():
    if sys.argv[1:2] == ["--blocks"]:
        chunks = [tuple(int(x) for x in c.split(",")) for c in (sys.argv[2:] or ["24,48"])]
        print(json.dumps({"constants": {"LINK_GBPS": LINK_GBPS, "XCHG_US": XCHG_US,
                                        "XCHG_HOST_US": XCHG_HOST_US},
                          "blocks": [dict(whole_px=w, **blocks_prediction(n, c, whole_px=w))
                                     for w in (2_200_000, 0) for c in chunks
                                     for n in (2, 4, 8)]}, indent=1), flush=True)
        return
    res = {"constants": {"LINK_GBPS": LINK_GBPS, "XCHG_US": XCHG_US,
                         "XCHG_HOST_US": XCHG_HOST_US},
           "resident_1080p_x8_ms": round(resident_ms(8), 3)}
    res["group_solve_ms"] = gs = group_solve_ms()
    res["stream"] = [stream_prediction(n, gs) for n in (1, 2, 4, 8)]
    res["bands"] = [bands_prediction(n) for n in (1, 2, 4, 8)]
    res["bands_no_whole"] = [bands_prediction(n, whole_px=0, overlap=False) for n in (2, 4, 8)]
    res["blocks"] = [blocks_prediction(n) for n in (2, 4, 8)]
    print(json.dumps(res, indent=1))


def link_table(rates=(25.0, 50.0, 100.0, 150.0)):
    """The stream leg's model at N = 1 and 8 for several link rates, from the
    committed batch solve times (frame_parallel.GROUP_SOLVE_MS; CPU only):
    how much the measured link (bench.stream_leg, link_gbps_measured) can
    move config 4's scaling."""
    base = stream_prediction(1, fp.GROUP_SOLVE_MS)
    out = []
    for r in rates:
        p8 = stream_prediction(8, fp.GROUP_SOLVE_MS, link_gbps=r)
        p8["speedup_vs_n1"] = round(p8["pairs_per_s"] / base["pairs_per_s"], 2)
        out.append(p8)
    return {"n1": base, "n8_by_link": out}


if __name__ == "__main__":
    if sys.argv[1:] == ["--link-table"]:
        print(json.dumps(link_table(), indent=1))
    else:
        main()
