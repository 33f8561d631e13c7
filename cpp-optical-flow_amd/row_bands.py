"""Config 5 on several GPUs: ONE frame pair split into row bands.

BASELINE config 5 is a single 7680x4320 pair (fp16, 3-level pyramid, 1000
iterations per level) on 8 GPUs, and SURVEY §8(e) proposes a row-band
decomposition with a halo exchange -- the only place on this path where a
pair (not a stream of pairs) is shared, so the only real exchange step.

Scheme (per pyramid level l, coarsest first):
  * every rank holds both frames and builds the full pyramid (K0; cheap);
  * rank r owns rows [a, b) of the level, and works on its *extended* band
    [a - H, b + H) (clipped to the image) as if it were a whole image: K1
    gradients and K2 iterations through the ordinary C ABI on row views;
  * iterations run in chunks of `chunk`; after every chunk each rank sends
    its first / last H owned rows of (u, v) to the neighbours, which store
    them in their halo rows (torch.distributed point-to-point, RCCL over
    xGMI on the GPU box);
  * H = chunk * max(A, AR) (A = window anchor): whatever is wrong at the
    extended band's edges (zero padding beyond it, reflect-101 in its K1)
    moves at most max(A, AR) rows per iteration, so after a chunk it has
    reached only halo rows, which the exchange then overwrites;
  * the finer level's warm start u = 2 u_c(y/2, x/2) (KU) reads coarse rows
    inside the coarse extended band, valid after the level's last exchange;
    band boundaries are multiples of 2^(levels-1), so every level's bands
    nest exactly;
  * finally rank 0 gathers the owned rows of (u, v).

Because K2's per-pixel operation sequence does not depend on how the image
is tiled or how iterations are split over launches, every owned row is
BIT-IDENTICAL to the single-GPU hsflow_flow_pyramid_device result (the
tests check exactly that; with the float64 oracle as the band solver the
same holds against oracle.flow_pyramid).

The solver is written against two small interfaces so that one code path
serves production and tests: `ops` (DeviceOps = libhsflow on torch CUDA
tensors; tests supply an oracle-backed one) and `comm` (DistComm =
torch.distributed; LocalComm = N virtual ranks in one process).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np


@dataclass(frozen=True)
class Band:
    a: int   # owned rows [a, b)
    b: int
    e0: int  # extended rows [e0, e1): owned + halo, clipped to the level
    e1: int


@dataclass(frozen=True)
class Plan:
    rows: int
    cols: int
    levels: int
    world: int
    window: int
    chunk: int
    halo: int
    sizes: tuple          # (rows_l, cols_l) per level
    bands: tuple          # bands[l][rank]


def anchors(window: int):
    A = window - window // 2 - 1  # hornSchunck.cpp:54, anchor of the box
    return A, window - 1 - A


def plan(rows: int, cols: int, levels: int, world: int, window: int, chunk: int) -> Plan:
    """Row bands for every level.  Raises ValueError if a band at some level
    would be shorter than the halo (too many ranks for the image)."""
    if world < 1 or levels < 1 or chunk < 1:
        raise ValueError("world, levels and chunk must be >= 1")
    A, AR = anchors(window)
    H = chunk * max(A, AR, 1)
    H += H & 1                      # even: extended bands start on even rows
    # nested bands on every level, each starting on an even row (even at the
    # coarsest level): the Jacobi kernels add the vertical window sums in an
    # order fixed by image-row parity, so a band solved as its own plane
    # must keep that parity to stay bit-identical to the whole-frame solve
    align = 1 << levels
    sizes = [(rows, cols)]
    for _ in range(1, levels):
        r, c = sizes[-1]
        sizes.append(((r + 1) // 2, (c + 1) // 2))
    cuts = [0] + [min(rows, int(round(k * rows / world / align)) * align)
                  for k in range(1, world)] + [rows]
    bands = []
    for l, (R, _) in enumerate(sizes):
        lv = []
        for r in range(world):
            a = cuts[r] >> l
            b = R if r == world - 1 else cuts[r + 1] >> l
            if world > 1 and b - a < H:
                raise ValueError(f"level {l}: band {r} has {b - a} rows < halo {H}; "
                                 "use fewer ranks or a shorter chunk")
            lv.append(Band(a, b, max(0, a - H) if r > 0 else 0,
                           min(R, b + H) if r < world - 1 else R))
        bands.append(tuple(lv))
    return Plan(rows, cols, levels, world, window, chunk, H, tuple(sizes), tuple(bands))


# --------------------------------------------------------------------- ops
class DeviceOps:
    """libhsflow on torch CUDA tensors (the product path)."""

    def __init__(self, window: int, alpha: float, device, stream=None):
        import torch
        import hsflow
        self.hs, self.torch = hsflow, torch
        self.window, self.alpha, self.device, self.stream = window, alpha, device, stream
        self._ws = None

    def levels(self, I0, I1, L: int):
        P0, P1 = self.hs.pyramid_build_device(I0, I1, L, stream=self.stream)
        return [I0] + P0, [I1] + P1

    def zeros(self, r: int, c: int):
        return self.torch.zeros((r, c), dtype=self.torch.float32, device=self.device)

    def workspace(self, r: int, c: int):
        need = self.hs.workspace_bytes(r, c, 1)
        if self._ws is None or self._ws.numel() < need:
            self._ws = self.torch.empty(need, dtype=self.torch.uint8, device=self.device)
        return self._ws

    def gradients(self, J0, J1):
        r, c = J0.shape
        ws = self.workspace(r, c)
        self.hs.gradients_device(J0, J1, ws, stream=self.stream)
        return ws

    def jacobi(self, ws, u, v, n: int):
        r, c = u.shape
        self.hs.jacobi_device(r, c, 1, self.window, n, self.alpha, u, v, ws,
                              warm_start=True, stream=self.stream)

    def upflow(self, uc, vc, u, v):
        self.hs.upflow_device(uc, vc, u, v, stream=self.stream)

    def set_zero(self, x):
        x.zero_()

    # overlapped schedule (solve_overlapped): the interior runs on a side
    # stream, the edge strips and the exchange on the caller's stream
    def clone(self, x):
        return x.clone()

    def cat_rows(self, a, b):
        return self.torch.cat([a, b], 0)

    def copy_rows(self, dst, src):
        dst.copy_(src)

    def _main(self):
        return self.torch.cuda.current_stream(self.device) if self.stream is None else self.stream

    def fork(self):
        if not hasattr(self, "_side"):
            self._side = self.torch.cuda.Stream(device=self.device)
        self._side.wait_stream(self._main())

    def jacobi_side(self, ws, u, v, n: int):
        r, c = u.shape
        self.hs.jacobi_device(r, c, 1, self.window, n, self.alpha, u, v, ws,
                              warm_start=True, stream=self._side)

    def join(self):
        self._main().wait_stream(self._side)


# -------------------------------------------------------------------- comm
class LocalComm:
    """N virtual ranks in one process (tests, one-GPU rehearsal): the halo
    exchange is a copy between the ranks' planes."""

    def start(self, states: Sequence["RankState"], level: int):
        self.exchange(states, level)
        return None

    def wait(self, handle):
        pass

    def exchange(self, states: Sequence["RankState"], level: int):
        p = states[0].plan
        H = p.halo
        for r in range(p.world - 1):
            up, dn = states[r], states[r + 1]
            bu, bd = p.bands[level][r], p.bands[level][r + 1]
            for fu, fd in ((up.u[level], dn.u[level]), (up.v[level], dn.v[level])):
                fd[bd.a - H:bd.a] = fu[bu.b - H:bu.b]   # r's bottom rows -> r+1's top halo
                fu[bu.b:bu.b + H] = fd[bd.a:bd.a + H]   # r+1's top rows -> r's bottom halo


class DistComm:
    """torch.distributed point-to-point (RCCL for CUDA tensors under the
    "nccl" backend; numpy / CPU tensors under "gloo")."""

    def exchange(self, states: Sequence["RankState"], level: int):
        self.wait(self.start(states, level))

    def wait(self, handle):
        for req in handle or ():
            req.wait()

    def start(self, states: Sequence["RankState"], level: int):
        """Post the halo exchange; returns the requests (wait() completes
        them: a stream wait under RCCL, a host wait under gloo)."""
        import torch
        import torch.distributed as dist
        (s,) = states
        p, r, H = s.plan, s.rank, s.plan.halo
        band = p.bands[level][r]
        ops = []

        def t(x):
            return torch.from_numpy(x) if isinstance(x, np.ndarray) else x
        # send copies: the overlapped schedule rewrites the owned rows (its
        # next interior solve) while a send may still be reading them
        for f in (s.u[level], s.v[level]):
            if r > 0:
                ops.append(dist.P2POp(dist.isend, t(f[band.a:band.a + H]).clone(), r - 1))
                ops.append(dist.P2POp(dist.irecv, t(f[band.a - H:band.a]), r - 1))
            if r < p.world - 1:
                ops.append(dist.P2POp(dist.isend, t(f[band.b - H:band.b]).clone(), r + 1))
                ops.append(dist.P2POp(dist.irecv, t(f[band.b:band.b + H]), r + 1))
        return dist.batch_isend_irecv(ops) if ops else []


# ------------------------------------------------------------------ solver
class RankState:
    def __init__(self, plan_: Plan, rank: int, ops):
        self.plan, self.rank, self.ops = plan_, rank, ops
        self.P0 = self.P1 = None
        self.u: List = [None] * plan_.levels
        self.v: List = [None] * plan_.levels


def solve(I0s, I1s, p: Plan, iters: int, ops_list, comm, ranks: Sequence[int]):
    """Run the banded coarse-to-fine solve for the given local ranks
    (one rank per process with DistComm; all ranks with LocalComm).
    I0s/I1s: each rank's copy of the full frames.  Returns the RankStates
    (level-0 owned rows of u/v are the result)."""
    states = [RankState(p, r, ops) for r, ops in zip(ranks, ops_list)]
    for s, I0, I1 in zip(states, I0s, I1s):
        s.P0, s.P1 = s.ops.levels(I0, I1, p.levels)
    for l in range(p.levels - 1, -1, -1):
        R, C = p.sizes[l]
        handles = []
        for s in states:
            bd = p.bands[l][s.rank]
            s.u[l], s.v[l] = s.ops.zeros(R, C), s.ops.zeros(R, C)
            if l < p.levels - 1:
                c0 = bd.e0 // 2                        # e0 is even (plan)
                c1 = min(p.sizes[l + 1][0], (bd.e1 + 1) // 2)
                s.ops.upflow(s.u[l + 1][c0:c1], s.v[l + 1][c0:c1],
                             s.u[l][bd.e0:bd.e1], s.v[l][bd.e0:bd.e1])
            handles.append(s.ops.gradients(s.P0[l][bd.e0:bd.e1], s.P1[l][bd.e0:bd.e1]))
        done = 0
        while True:
            n = min(p.chunk, iters - done)
            if n > 0:
                for s, h in zip(states, handles):  # each rank owns its ops/workspace
                    bd = p.bands[l][s.rank]
                    s.ops.jacobi(h, s.u[l][bd.e0:bd.e1], s.v[l][bd.e0:bd.e1], n)
                done += n
            if p.world > 1:
                comm.exchange(states, l)
            if done >= iters:
                break
        for s in states:
            if l + 1 < p.levels:
                s.u[l + 1] = s.v[l + 1] = None     # coarse level no longer needed
    return states


def _clone(ops, x):
    if hasattr(ops, "clone"):
        return ops.clone(x)
    return x if isinstance(x, tuple) else x.copy()  # numpy (oracle-backed ops)


def _cat(ops, a, b):
    return ops.cat_rows(a, b) if hasattr(ops, "cat_rows") else np.concatenate([a, b], 0)


def _copy(ops, dst, src):
    if hasattr(ops, "copy_rows"):
        ops.copy_rows(dst, src)
    else:
        dst[...] = src


def overlap_ok(p: Plan) -> bool:
    """The overlapped schedule needs every band to hold two halos of rows
    (its edge strips' valid rows and the interior's must tile the band)."""
    return p.world > 1 and all(bd.b - bd.a >= 2 * p.halo for lv in p.bands for bd in lv)


def solve_overlapped(I0s, I1s, p: Plan, iters: int, ops_list, comm, ranks: Sequence[int]):
    """solve() with each chunk's halo exchange hidden behind the next
    chunk's interior iterations.  Per rank and chunk, with H = p.halo and the
    owned rows [a, b):
      * the interior [a, b) is solved in place as its own plane: its edges at
        a and b are artificial, so after the chunk its rows [a + H, b - H) are
        exact -- and it needs nothing from the neighbours, so it runs (on a
        side stream on the GPU) while the previous chunk's exchange is in
        flight;
      * the edge strips [a - H, a + 2H) and [b - 2H, b + H) -- the received
        halo rows plus a snapshot of the owned rows taken before the interior
        overwrites them -- are solved once the exchange has landed, on the
        caller's stream, concurrently with the interior; their middle thirds
        are the exact rows [a, a + H) and [b - H, b), written back (after
        the interior has finished) and sent to the neighbours as copies
        (posted, not waited for: the next interior solve may rewrite the
        rows while a send is still reading).
    Critical path per chunk: max(interior, exchange + strip) instead of
    band + exchange.  Every sub-plane starts on an even image row (H and the
    band starts are even), so every owned row is BIT-IDENTICAL to solve()
    and to the undivided solve.  Gradients of the three sub-planes are
    computed once per level (their artificial edges differ from the band's)."""
    if not overlap_ok(p):
        raise ValueError("overlapped schedule needs world > 1 and bands of >= 2 halos")
    H = p.halo
    states = [RankState(p, r, ops) for r, ops in zip(ranks, ops_list)]
    for s, I0, I1 in zip(states, I0s, I1s):
        s.P0, s.P1 = s.ops.levels(I0, I1, p.levels)

    for l in range(p.levels - 1, -1, -1):
        R, C = p.sizes[l]
        g = []
        for s in states:
            bd = p.bands[l][s.rank]
            s.u[l], s.v[l] = s.ops.zeros(R, C), s.ops.zeros(R, C)
            if l < p.levels - 1:
                c0 = bd.e0 // 2
                c1 = min(p.sizes[l + 1][0], (bd.e1 + 1) // 2)
                s.ops.upflow(s.u[l + 1][c0:c1], s.v[l + 1][c0:c1],
                             s.u[l][bd.e0:bd.e1], s.v[l][bd.e0:bd.e1])
            top = bd.a > 0
            bot = bd.b < R
            # DeviceOps computes gradients into one reused workspace: each
            # sub-plane keeps its own copy (which also holds its solve's
            # ping-pong planes, so interior and strips can run concurrently)
            gi = _clone(s.ops, s.ops.gradients(s.P0[l][bd.a:bd.b], s.P1[l][bd.a:bd.b]))
            gt = _clone(s.ops, s.ops.gradients(s.P0[l][bd.a - H:bd.a + 2 * H],
                                               s.P1[l][bd.a - H:bd.a + 2 * H])) if top else None
            gb = _clone(s.ops, s.ops.gradients(s.P0[l][bd.b - 2 * H:bd.b + H],
                                               s.P1[l][bd.b - 2 * H:bd.b + H])) if bot else None
            g.append((gi, gt, gb, top, bot))
        pending = None
        done = 0
        while done < iters:
            n = min(p.chunk, iters - done)
            snaps = []
            for s, (gi, gt, gb, top, bot) in zip(states, g):
                bd = p.bands[l][s.rank]
                u, v = s.u[l], s.v[l]
                # the owned rows the strips need, before the interior moves on
                snaps.append((_clone(s.ops, u[bd.a:bd.a + 2 * H]) if top else None,
                              _clone(s.ops, v[bd.a:bd.a + 2 * H]) if top else None,
                              _clone(s.ops, u[bd.b - 2 * H:bd.b]) if bot else None,
                              _clone(s.ops, v[bd.b - 2 * H:bd.b]) if bot else None))
                if hasattr(s.ops, "fork"):  # interior on the side stream
                    s.ops.fork()
                    s.ops.jacobi_side(gi, u[bd.a:bd.b], v[bd.a:bd.b], n)
                else:
                    s.ops.jacobi(gi, u[bd.a:bd.b], v[bd.a:bd.b], n)
            comm.wait(pending)                                     # chunk - 1's halos
            strips = []
            for s, (gi, gt, gb, top, bot), (tu, tv, bu, bv) in zip(states, g, snaps):
                bd = p.bands[l][s.rank]
                u, v = s.u[l], s.v[l]
                st = sb = None
                if top:
                    st = (_cat(s.ops, u[bd.a - H:bd.a], tu), _cat(s.ops, v[bd.a - H:bd.a], tv))
                    s.ops.jacobi(gt, st[0], st[1], n)
                if bot:
                    sb = (_cat(s.ops, bu, u[bd.b:bd.b + H]), _cat(s.ops, bv, v[bd.b:bd.b + H]))
                    s.ops.jacobi(gb, sb[0], sb[1], n)
                strips.append((st, sb))
            for s, (st, sb) in zip(states, strips):
                bd = p.bands[l][s.rank]
                u, v = s.u[l], s.v[l]
                if hasattr(s.ops, "join"):
                    s.ops.join()
                if st is not None:
                    _copy(s.ops, u[bd.a:bd.a + H], st[0][H:2 * H])
                    _copy(s.ops, v[bd.a:bd.a + H], st[1][H:2 * H])
                if sb is not None:
                    _copy(s.ops, u[bd.b - H:bd.b], sb[0][H:2 * H])
                    _copy(s.ops, v[bd.b - H:bd.b], sb[1][H:2 * H])
            pending = comm.start(states, l)
            done += n
        comm.wait(pending)
        for s in states:
            if l + 1 < p.levels:
                s.u[l + 1] = s.v[l + 1] = None
    return states


def gather_owned(states, p: Plan, comm):
    """Rank 0 assembles level 0 from every rank's owned rows.  With LocalComm
    all states are local; with DistComm every rank calls this (rank 0 gets
    the arrays, others None)."""
    if isinstance(comm, LocalComm):
        def copy(x):
            return x.clone() if hasattr(x, "clone") else x.copy()
        u, v = copy(states[0].u[0]), copy(states[0].v[0])
        for s in states:
            bd = p.bands[0][s.rank]
            u[bd.a:bd.b] = s.u[0][bd.a:bd.b]
            v[bd.a:bd.b] = s.v[0][bd.a:bd.b]
        return u, v
    import torch
    import torch.distributed as dist
    (s,) = states
    bd = p.bands[0][s.rank]

    def t(x):
        return torch.from_numpy(x) if isinstance(x, np.ndarray) else x
    ops = []
    if s.rank == 0:
        for r in range(1, p.world):
            b = p.bands[0][r]
            for f in (s.u[0], s.v[0]):
                ops.append(dist.P2POp(dist.irecv, t(f[b.a:b.b]), r))
    else:
        for f in (s.u[0], s.v[0]):
            ops.append(dist.P2POp(dist.isend, t(f[bd.a:bd.b]), 0))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return (s.u[0], s.v[0]) if s.rank == 0 else (None, None)
