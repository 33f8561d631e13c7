"""Frame-parallel driver: a stream of frame pairs sharded across ranks.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on
MI355X, "gloo" for CPU tests).  Frame pairs are independent, so the only
communication is moving data: rank 0 holds the stream, scatters pair j to
rank j % world (point-to-point send/recv, batched; RCCL has no scatter
primitive), every rank solves its pairs with libhsflow, and (u, v) are
gathered back to rank 0 in stream order.  No reduction touches the hot path.

The reference has no distributed code: this is the north_star's
config 4 ("64 synthetic 1080p pairs sharded one-per-GPU, RCCL
scatter/gather").  The per-pair solver is injected (`solve`), so the
protocol is exercised with gloo + CPU tensors in tests while production uses
hsflow.flow_device on the GPU.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

Pair = Tuple[torch.Tensor, torch.Tensor]


def _fence(tensors) -> None:
    """gloo moves CUDA tensors with host code, not in stream order: the
    stream that wrote them must have finished before they are posted
    (RCCL is stream-ordered and needs nothing; row_bands.host_transport_fence)."""
    cuda = [t for t in tensors if isinstance(t, torch.Tensor) and t.is_cuda]
    if cuda and dist.get_backend() != "nccl":
        torch.cuda.current_stream(cuda[0].device).synchronize()


def owner(j: int, world: int) -> int:
    """Rank that solves pair j (round-robin, weak-scales with world)."""
    return j % world


def my_pairs(n_pairs: int, rank: int, world: int) -> List[int]:
    return [j for j in range(n_pairs) if owner(j, world) == rank]


def scatter_pairs(stream: Optional[Sequence[Pair]], n_pairs: int, shape, dtype, device,
                  rank: int, world: int) -> List[Pair]:
    """Rank 0 sends pair j to owner(j); returns this rank's pairs in order.
    `stream` is only read on rank 0."""
    mine = my_pairs(n_pairs, rank, world)
    if world == 1:
        return [(stream[j][0].to(device), stream[j][1].to(device)) for j in mine]
    ops, out = [], []
    if rank == 0:
        for j in range(n_pairs):
            dst = owner(j, world)
            if dst == 0:
                continue
            I0, I1 = stream[j]
            ops.append(dist.P2POp(dist.isend, I0.to(device).contiguous(), dst))
            ops.append(dist.P2POp(dist.isend, I1.to(device).contiguous(), dst))
        out = [(stream[j][0].to(device), stream[j][1].to(device)) for j in mine]
        _fence([op.tensor for op in ops])
    else:
        for _ in mine:
            a = torch.empty(shape, dtype=dtype, device=device)
            b = torch.empty(shape, dtype=dtype, device=device)
            ops.append(dist.P2POp(dist.irecv, a, 0))
            ops.append(dist.P2POp(dist.irecv, b, 0))
            out.append((a, b))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return out


def gather_flows(flows: List[Pair], n_pairs: int, shape, device, rank: int,
                 world: int) -> Optional[List[Pair]]:
    """Inverse of scatter_pairs for the (u, v) results; rank 0 returns the
    full list in stream order, other ranks None."""
    mine = my_pairs(n_pairs, rank, world)
    if world == 1:
        return list(flows)
    ops = []
    result: List[Optional[Pair]] = [None] * n_pairs
    if rank == 0:
        for k, j in enumerate(mine):
            result[j] = flows[k]
        for j in range(n_pairs):
            src = owner(j, world)
            if src == 0:
                continue
            u = torch.empty(shape, dtype=torch.float32, device=device)
            v = torch.empty(shape, dtype=torch.float32, device=device)
            ops.append(dist.P2POp(dist.irecv, u, src))
            ops.append(dist.P2POp(dist.irecv, v, src))
            result[j] = (u, v)
    else:
        for (u, v) in flows:
            ops.append(dist.P2POp(dist.isend, u.contiguous(), 0))
            ops.append(dist.P2POp(dist.isend, v.contiguous(), 0))
        _fence([op.tensor for op in ops])
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return result if rank == 0 else None


def run_stream(stream: Optional[Sequence[Pair]], n_pairs: int, shape, dtype,
               solve: Callable[[torch.Tensor, torch.Tensor], Pair], device,
               rank: int, world: int, gather: bool = True):
    """Scatter -> solve every owned pair -> gather.  Returns rank 0's list of
    (u, v) in stream order (None elsewhere, or when gather=False)."""
    pairs = scatter_pairs(stream, n_pairs, shape, dtype, device, rank, world)
    flows = [solve(I0, I1) for (I0, I1) in pairs]
    if not gather:
        return None
    return gather_flows(flows, n_pairs, shape, device, rank, world)


def chunk_split(mine: Sequence[int], chunks: int) -> List[List[int]]:
    """This rank's pairs cut into at most `chunks` contiguous groups (sizes
    differ by at most one, larger groups first; no empty groups)."""
    n = len(mine)
    k = max(1, min(chunks, n)) if n else 0
    out, start = [], 0
    for c in range(k):
        size = n // k + (1 if c < n % k else 0)
        out.append(list(mine[start:start + size]))
        start += size
    return out


def size_split(mine: Sequence[int], sizes: Sequence[int]) -> List[List[int]]:
    """This rank's pairs cut into consecutive groups of the given sizes."""
    assert sum(sizes) == len(mine) and all(s > 0 for s in sizes), (sizes, len(mine))
    out, start = [], 0
    for s in sizes:
        out.append(list(mine[start:start + s]))
        start += s
    return out


# ---- group sizes of the pipelined stream (BASELINE config 4) -------------
# Solve time of a batch of g 1080p pairs (300 iterations, w 5), g = 1..8, on
# one MI355X (eager calls as the stream leg makes them, clocks settled;
# scripts/scale_predict.py `group_solve_ms`, profiles/r05_scale_prediction.json):
# small batches leave most of the chip idle, so a pair costs 0.72 ms alone
# and 0.46 ms in a batch of 8.
GROUP_SOLVE_MS = (0.7220, 1.2672, 1.9887, 2.3102, 2.6177, 2.9458, 3.4142, 3.6790)
# RCCL point-to-point per peer link (one xGMI link each way; an assumption
# of a third of the link's 153 GB/s: DESIGN.md §6).  Only the fallback: the
# stream leg measures the link before its timed passes (measure_link_gbps)
# and sizes its groups with that rate.
LINK_GBPS = 50.0


def measure_link_gbps(device, rank: int, world: int, nbytes: int, reps: int = 3) -> dict:
    """The point-to-point rate of rank 0's link to every peer, measured with
    the transport the stream uses: per peer, `reps` round trips of one
    `nbytes` buffer (0 -> peer -> 0; the peers take turns, the others idle),
    rate = nbytes / (best round trip / 2).  Rank 0 broadcasts the result, so
    every rank sizes its groups (group_sizes) with the same value: the
    slowest peer's rate (`link_gbps`), or LINK_GBPS if a measurement is not
    finite and positive, clamped to [1, 1000] for the model.  Returns
    {"link_gbps" (the model's input), "measured_gbps", "per_peer"} on every
    rank.
    Runs outside any timed region; one call costs ~2 reps (world - 1)
    transfers of nbytes (7 peers x 3 x 2 x 8.3 MB at 50 GB/s: ~7 ms)."""
    import time
    per_peer: List[float] = []
    if world > 1:
        buf = torch.empty(max(1, nbytes // 4), dtype=torch.float32, device=device)
        buf.fill_(1.0)
        sync = ((lambda: torch.cuda.synchronize(device)) if buf.is_cuda else (lambda: None))
        for peer in range(1, world):
            best = float("inf")
            for it in range(reps + 1):  # the first round trip warms the path
                dist.barrier()
                if rank == 0:
                    sync()
                    t0 = time.perf_counter()
                    _fence([buf])
                    dist.send(buf, peer)
                    dist.recv(buf, peer)
                    sync()
                    if it > 0:
                        best = min(best, time.perf_counter() - t0)
                elif rank == peer:
                    dist.recv(buf, 0)
                    sync()
                    dist.send(buf, 0)
                    sync()
            if rank == 0:
                per_peer.append(buf.numel() * 4 / (best / 2) / 1e9 if best > 0 else 0.0)
        val = torch.tensor([min(per_peer) if per_peer else LINK_GBPS], dtype=torch.float64)
        if dist.get_backend() == "nccl":
            val = val.to(device)
        dist.broadcast(val, 0)
        rate = float(val.item())
    else:
        rate = LINK_GBPS
    if not (rate > 0.0 and rate < float("inf")):
        rate = LINK_GBPS
    # the schedule model's input stays within [1, 1000] GB/s (a host-side
    # transport such as gloo over CUDA tensors measures ~0.03 GB/s, at which
    # the model would cut every share into single pairs)
    return {"link_gbps": min(max(rate, 1.0), 1000.0), "measured_gbps": rate,
            "per_peer": [round(x, 3) for x in per_peer]}


def pipeline_ms(sizes: Sequence[int], in_mb: float, out_mb: float,
                solve_ms: Sequence[float] = GROUP_SOLVE_MS, link_gbps: float = LINK_GBPS,
                remote: bool = True) -> float:
    """Modelled time of one rank's share in groups of `sizes`: group c's
    frames arrive over the link (all groups posted at once, in order), its
    solve starts when they have arrived and the previous solve is done, its
    (u, v) go back over the other direction of the link in order.  in_mb /
    out_mb: MB per pair each way.  remote = False: rank 0's own share (no
    transfers)."""
    arrive = solve_end = home = 0.0
    for g in sizes:
        ms = solve_ms[g - 1] if g <= len(solve_ms) else solve_ms[-1] * g / len(solve_ms)
        if remote:
            arrive += g * in_mb / link_gbps
        solve_end = max(arrive, solve_end) + ms
        home = max(home, solve_end) + (g * out_mb / link_gbps if remote else 0.0)
    return max(home, solve_end)


def _partitions(n: int, cap: int):
    """Non-increasing sequences of parts <= cap summing to n."""
    if n == 0:
        yield ()
        return
    for first in range(min(n, cap), 0, -1):
        for rest in _partitions(n - first, first):
            yield (first,) + rest


def group_sizes(share: int, world: int, in_mb: float, out_mb: float,
                solve_ms: Sequence[float] = GROUP_SOLVE_MS, link_gbps: float = LINK_GBPS,
                cap: int = 8) -> List[int]:
    """Group sizes of a rank's share of the stream (the same on every rank,
    so each end of a link knows the other's grouping).  One rank: batches of
    at most `cap` pairs (8 pairs fill the chip; larger batches fall out of
    the Infinity Cache).  Several ranks: the non-increasing sizes <= cap
    that minimise pipeline_ms -- a large first group solves efficiently
    while later groups arrive, small last groups keep the exposed return of
    the last (u, v) short."""
    if share <= 0:
        return []
    if world == 1:
        k = -(-share // cap)
        return [share // k + (1 if c < share % k else 0) for c in range(k)]
    best = None
    for sizes in _partitions(share, cap):
        t = pipeline_ms(sizes, in_mb, out_mb, solve_ms, link_gbps)
        if best is None or t < best[0] - 1e-9:
            best = (t, list(sizes))
    return best[1]


def batch_of(frames: Sequence[torch.Tensor], device) -> torch.Tensor:
    """The frames as one (len, rows, cols) batch: a view when they already
    lie back to back in one device buffer (a stream decoded into one
    allocation, as bench.py holds it), else a stacked copy."""
    f0 = frames[0]
    if f0.device == torch.device(device) and all(f.is_contiguous() for f in frames):
        step = f0.numel() * f0.element_size()
        base = f0.untyped_storage().data_ptr()
        if all(f.untyped_storage().data_ptr() == base and
               f.data_ptr() == f0.data_ptr() + k * step and f.shape == f0.shape
               and f.dtype == f0.dtype for k, f in enumerate(frames)):
            return f0.as_strided((len(frames),) + tuple(f0.shape),
                                 (f0.numel(),) + tuple(f0.stride()))
    return torch.stack([f.to(device) for f in frames])


def run_stream_pipelined(stream: Optional[Sequence[Pair]], n_pairs: int, shape, dtype,
                         solve_batch: Callable[[torch.Tensor, torch.Tensor], Pair], device,
                         rank: int, world: int, chunks: int = 2, gather: bool = True,
                         sizes: Optional[Callable[[int], Sequence[int]]] = None):
    """run_stream with the transfers overlapped: each rank's share is cut into
    groups (`sizes(share)` gives their sizes, the same function on every
    rank; default `chunks` near-equal groups); rank 0 posts the scatter of
    every group at once, a rank solves group c (one batched call) as soon as
    group c has arrived -- group c+1 is still in flight -- and sends group
    c's (u, v) back, one message per plane, while it solves group c+1.  With
    RCCL every step is stream-ordered: work.wait() makes the compute stream
    wait on the communicator's stream, so no host blocking until rank 0
    collects the result.

    The point-to-point calls are issued in the same order on both ends of
    every link (all scatter groups, then the gather groups in group order),
    one batch per group on both ends (rank 0's batch of group c spans every
    destination), which is what keeps RCCL's in-order per-peer matching free
    of deadlock: a rank posts its receives for every group before its first
    result send.  (Verified with gloo, world 2 and 3; the
    RCCL schedule runs first on the driver's multi-GPU node.)
    Frames travel in their own dtype (the bench holds the stream as u8, the
    type main.cpp:13-14 leaves the frames in: a quarter of f32's bytes).
    Returns rank 0's (u, v) list in stream order (None elsewhere, or when
    gather=False).  Bit-identical to run_stream: only the schedule changes."""
    mine = my_pairs(n_pairs, rank, world)

    def split(r, pairs):
        if sizes is None:
            return chunk_split(pairs, chunks)
        return size_split(pairs, list(sizes(len(pairs))))

    if world == 1:
        out: List[Pair] = []
        for grp in split(0, mine):
            I0 = batch_of([stream[j][0] for j in grp], device)
            I1 = batch_of([stream[j][1] for j in grp], device)
            u, v = solve_batch(I0, I1)
            out.extend((u[k], v[k]) for k in range(len(grp)))
        return out if gather else None
    groups = {r: split(r, my_pairs(n_pairs, r, world)) for r in range(world)}
    n_groups = max(len(g) for g in groups.values())
    # 1. scatter: every group of every rank posted up front, group-major;
    #    one batch per group holding the sends to EVERY destination, so the
    #    group travels over all of rank 0's links at once (a batch per
    #    destination would queue the destinations one after another on the
    #    communicator's stream: 7 x 1.3 ms before the last rank of 8 could
    #    start).  Point-to-point calls match in order per peer, whatever the
    #    batching on the other side (each receiver posts one batch per group)
    recv_groups: List[Tuple[torch.Tensor, torch.Tensor, list]] = []
    if rank == 0:
        scatter_reqs = []
        for c in range(n_groups):
            ops = []
            for dst in range(1, world):
                if c >= len(groups[dst]):
                    continue
                for j in groups[dst][c]:
                    I0, I1 = stream[j]
                    ops.append(dist.P2POp(dist.isend, I0.to(device).contiguous(), dst))
                    ops.append(dist.P2POp(dist.isend, I1.to(device).contiguous(), dst))
            if ops:
                # fenced after the send tensors exist: a .to() / .contiguous()
                # that really copies is queued before gloo reads the buffer
                # (as scatter_pairs does)
                _fence([op.tensor for op in ops])
                scatter_reqs.extend(dist.batch_isend_irecv(ops))
    else:
        for grp in groups[rank]:
            a = torch.empty((len(grp),) + tuple(shape), dtype=dtype, device=device)
            b = torch.empty((len(grp),) + tuple(shape), dtype=dtype, device=device)
            ops = []
            for k in range(len(grp)):
                ops.append(dist.P2POp(dist.irecv, a[k], 0))
                ops.append(dist.P2POp(dist.irecv, b[k], 0))
            recv_groups.append((a, b, dist.batch_isend_irecv(ops)))
    # 2. per group: solve, then ship the result (rank 0 posts its receives
    #    of the remote ranks' group c first, so they need not wait behind
    #    its own solve of group c on the communicator's stream); a group's
    #    (u, v) travel as two messages, one per plane batch
    result: List[Optional[Pair]] = [None] * n_pairs
    pending = []
    for c in range(n_groups):
        if rank == 0 and gather:  # posted before rank 0's own solve c
            ops = []
            for src in range(1, world):
                if c >= len(groups[src]):
                    continue
                grp = groups[src][c]
                u = torch.empty((len(grp),) + tuple(shape), dtype=torch.float32, device=device)
                v = torch.empty_like(u)
                ops.append(dist.P2POp(dist.irecv, u, src))
                ops.append(dist.P2POp(dist.irecv, v, src))
                for k, j in enumerate(grp):
                    result[j] = (u[k], v[k])
            if ops:
                pending.append((None, None, dist.batch_isend_irecv(ops)))
        if c < len(groups[rank]):
            grp = groups[rank][c]
            if rank == 0:
                I0 = batch_of([stream[j][0] for j in grp], device)
                I1 = batch_of([stream[j][1] for j in grp], device)
            else:
                I0, I1, reqs = recv_groups[c]
                for req in reqs:
                    req.wait()
            u, v = solve_batch(I0, I1)
            if rank == 0:
                for k, j in enumerate(grp):
                    result[j] = (u[k], v[k])
            elif gather:
                u, v = u.contiguous(), v.contiguous()
                _fence([u, v])
                ops = [dist.P2POp(dist.isend, u, 0), dist.P2POp(dist.isend, v, 0)]
                pending.append((u, v, dist.batch_isend_irecv(ops)))
    if rank == 0:
        for req in scatter_reqs:
            req.wait()
    for _, _, reqs in pending:
        for req in reqs:
            req.wait()
    if not gather:
        return None
    return result if rank == 0 else None


def max_over_ranks(seconds: float, device, world: int) -> float:
    """The bench's timing rule: the slowest rank defines the step time."""
    if world == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
