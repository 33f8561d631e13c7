"""Config 5 split over ranks (cpp-optical-flow_amd/row_bands.py): one frame
pair in row bands with a halo exchange after every chunk of iterations.

The claim under test is exactness: every owned row equals the undivided
solve bit for bit.  On CPU the band solver is the float64 oracle (test
infrastructure) and the reference is oracle.flow_pyramid; the exchange runs
both in-process (LocalComm) and over torch.distributed gloo with 2 and 3
processes (DistComm, the code RCCL runs on the GPU box).  On the GPU the
band solver is libhsflow and the reference hsflow.flow_pyramid_device."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
import row_bands as rb
from synth_ref import synth_pair


class OracleOps:
    """The band operations restated with the float64 oracle pieces."""

    def __init__(self, window, alpha):
        self.window, self.alpha = window, alpha

    def levels(self, I0, I1, L):
        a, b = np.asarray(I0, np.float64), np.asarray(I1, np.float64)
        rnd = oracle.integer_pair(a, b)
        P0, P1 = [a], [b]
        for _ in range(1, L):
            P0.append(oracle.pyrdown(P0[-1], rnd))
            P1.append(oracle.pyrdown(P1[-1], rnd))
        return P0, P1

    def zeros(self, r, c):
        return np.zeros((r, c), np.float64)

    def gradients(self, J0, J1):
        return oracle.gradients(J0, J1)

    def jacobi(self, g, u, v, n):
        nu, nv = oracle.jacobi(g[0], g[1], g[2], u, v, self.window, n, self.alpha)
        u[...] = nu
        v[...] = nv

    def upflow(self, uc, vc, u, v):
        r, c = u.shape
        u[...] = 2.0 * np.repeat(np.repeat(uc, 2, 0), 2, 1)[:r, :c]
        v[...] = 2.0 * np.repeat(np.repeat(vc, 2, 0), 2, 1)[:r, :c]


# ------------------------------------------------------------------ planning
@pytest.mark.parametrize("rows,levels,world,chunk", [(4320, 3, 8, 12), (1080, 3, 4, 6),
                                                     (97, 2, 3, 3), (64, 1, 2, 4)])
def test_plan_bands_tile_and_nest(rows, levels, world, chunk):
    p = rb.plan(rows, 77, levels, world, 5, chunk)
    assert p.halo == chunk * 2 and p.halo % 2 == 0
    for l, (R, _) in enumerate(p.sizes):
        bands = p.bands[l]
        assert bands[0].a == 0 and bands[-1].b == R
        for x, y in zip(bands, bands[1:]):
            assert x.b == y.a                               # owned rows tile the level
        for k, bd in enumerate(bands):
            assert bd.b - bd.a >= p.halo or world == 1
            assert bd.e0 == (0 if k == 0 else bd.a - p.halo)
            assert bd.e1 == (R if k == world - 1 else bd.b + p.halo)
            # even band starts: warm starts map rows exactly and the band keeps
            # image-row parity (the kernels' vertical summation order)
            assert bd.e0 % 2 == 0
            if l > 0:
                assert bd.a == p.bands[0][k].a >> l         # bands nest across levels


def test_plan_rejects_bands_shorter_than_the_halo():
    with pytest.raises(ValueError):
        rb.plan(100, 50, 3, 8, 5, 12)


# --------------------------------------------------- oracle-backed, one process
def _pair(rows, cols, seed=1000):
    return synth_pair(seed, rows, cols)


@pytest.mark.parametrize("world,levels,chunk,window", [(2, 2, 3, 5), (3, 3, 2, 5),
                                                       (4, 1, 2, 3), (2, 3, (2, 4), 5),
                                                       (3, 2, (1, 3), 5)])
def test_local_bands_equal_undivided_oracle(world, levels, chunk, window):
    I0, I1 = _pair(70, 53)
    iters = 7
    p = rb.plan(70, 53, levels, world, window, chunk)
    ops = [OracleOps(window, 1.0) for _ in range(world)]
    comm = rb.LocalComm()
    states = rb.solve([I0] * world, [I1] * world, p, iters, ops, comm, list(range(world)))
    u, v = rb.gather_owned(states, p, comm)
    uo, vo = oracle.flow_pyramid(I0, I1, levels, window, iters, 1.0)
    assert np.array_equal(u, uo) and np.array_equal(v, vo)


@pytest.mark.parametrize("world,levels,chunk,window,iters", [(2, 2, 3, 5, 7), (3, 1, 2, 5, 9),
                                                             (4, 2, 2, 3, 5), (2, 1, 3, 5, 3),
                                                             (2, 2, (2, 3), 5, 7)])
def test_local_overlapped_bands_equal_undivided_oracle(world, levels, chunk, window, iters):
    """The overlapped schedule (interior solved while the halos travel,
    edge strips solved from the received halos and a snapshot) gives the
    undivided solve's bits, like the plain schedule."""
    I0, I1 = _pair(101, 53)
    p = rb.plan(101, 53, levels, world, window, chunk)
    assert rb.overlap_ok(p)
    comm = rb.LocalComm()
    ops = [OracleOps(window, 1.0) for _ in range(world)]
    states = rb.solve_overlapped([I0] * world, [I1] * world, p, iters, ops, comm,
                                 list(range(world)))
    u, v = rb.gather_owned(states, p, comm)
    uo, vo = oracle.flow_pyramid(I0, I1, levels, window, iters, 1.0)
    assert np.array_equal(u, uo) and np.array_equal(v, vo)


def test_fit_plan_cuts_coarse_chunks_to_the_bands():
    """bench's --chunk 24,48 at 8 ranks: window 5 fits as asked; window 7's
    level-2 halo (144 rows) does not fit its 134-row bands, so that chunk is
    cut (and said); the overlapped schedule needs two halos per band, and a
    coarse level never ends with a halo below half the finer one's."""
    p, notes = rb.fit_plan(4320, 7680, 3, 8, 5, (24, 48))
    assert p.chunks == (24, 48, 48) and notes == []
    p, notes = rb.fit_plan(4320, 7680, 3, 8, 7, (24, 48))
    assert p.chunks[:2] == (24, 48) and p.chunks[2] < 48 and len(notes) == 1
    with pytest.raises(ValueError):
        rb.plan(4320, 7680, 3, 8, 7, (24, 48))
    p, notes = rb.fit_plan(4320, 7680, 3, 8, 5, (24, 48), overlap=True)
    assert rb.overlap_ok(p) and notes
    for w in (3, 5, 7, 9):
        for ov in (False, True):
            p, _ = rb.fit_plan(4320, 7680, 3, 8, w, (24, 48), overlap=ov)
            for l in range(2):
                assert p.halos[l + 1] >= p.halos[l] // 2 + 1
            assert not ov or rb.overlap_ok(p)
    # one rank: nothing to fit
    p, notes = rb.fit_plan(4320, 7680, 3, 1, 7, 1000)
    assert p.chunks == (1000,) * 3 and notes == []


def test_whole_levels_plan():
    """Coarse levels solved whole on every rank: extended band = the plane,
    no halo, ownership still split for the gather; a whole level's coarser
    levels must be whole too; the 8K pyramid at N = 8 takes level 2 whole."""
    assert rb.whole_levels(4320, 7680, 3, 8, 2_200_000) == (False, False, True)
    assert rb.whole_levels(4320, 7680, 3, 1, 2_200_000) == (False, False, False)
    p = rb.plan(400, 522, 3, 3, 5, 6, whole=(False, True, True))
    for l in (1, 2):
        R = p.sizes[l][0]
        assert p.halos[l] == 0
        assert all(bd.e0 == 0 and bd.e1 == R for bd in p.bands[l])
        assert [bd.a for bd in p.bands[l]] == sorted(bd.a for bd in p.bands[l])
        assert p.bands[l][-1].b == R
    with pytest.raises(ValueError):
        rb.plan(400, 522, 3, 3, 5, 6, whole=(False, True, False))


@pytest.mark.parametrize("world,whole", [(2, (False, True)), (3, (False, True))])
def test_local_bands_with_whole_levels_equal_undivided_oracle(world, whole):
    I0, I1 = synth_pair(1000, ROWS, COLS)
    p = rb.plan(ROWS, COLS, LEVELS, world, 5, CHUNK, whole=whole)
    for solve in (rb.solve, rb.solve_overlapped):
        if solve is rb.solve_overlapped and not rb.overlap_ok(p):
            continue
        states = solve([I0] * world, [I1] * world, p, ITERS,
                       [OracleOps(5, 1.0) for _ in range(world)], rb.LocalComm(),
                       list(range(world)))
        u, v = rb.gather_owned(states, p, rb.LocalComm())
        uo, vo = oracle.flow_pyramid(I0, I1, LEVELS, 5, ITERS, 1.0)
        assert np.array_equal(u, uo) and np.array_equal(v, vo)


def test_plan_per_level_chunks():
    """Longer chunks on coarse levels (the bench's 24 / 48): one halo per
    level; a coarse halo shorter than half the finer one is refused (the
    finer level's warm start reads coarse halo rows)."""
    p = rb.plan(4320, 7680, 3, 8, 5, (24, 48))
    assert p.chunks == (24, 48, 48) and p.halos == (48, 96, 96)
    assert p.chunk == 24 and p.halo == 48
    for l, lv in enumerate(p.bands):
        for k, bd in enumerate(lv):
            assert bd.e0 == (0 if k == 0 else bd.a - p.halos[l])
    with pytest.raises(ValueError):
        rb.plan(400, 60, 2, 2, 5, (24, 4))
    assert rb.level_chunks(7, 3) == (7, 7, 7)


def test_overlap_needs_two_halos_per_band():
    p = rb.plan(60, 30, 1, 3, 5, 6)   # bands of 20 rows, halo 12
    assert not rb.overlap_ok(p)
    with pytest.raises(ValueError):
        rb.solve_overlapped([None] * 3, [None] * 3, p, 4, [None] * 3, rb.LocalComm(), [0, 1, 2])
    assert not rb.overlap_ok(rb.plan(60, 30, 1, 1, 5, 2))   # nothing to overlap on one rank


def test_local_bands_non_integral_frames():
    I0, I1 = _pair(66, 41)
    I0 = I0 * np.float32(0.7) + np.float32(0.2)
    p = rb.plan(66, 41, 2, 2, 5, 3)
    comm = rb.LocalComm()
    states = rb.solve([I0] * 2, [I1] * 2, p, 5, [OracleOps(5, 1.0) for _ in range(2)], comm,
                      [0, 1])
    u, _ = rb.gather_owned(states, p, comm)
    uo, _ = oracle.flow_pyramid(I0, I1, 2, 5, 5, 1.0)
    assert np.array_equal(u, uo)


# ------------------------------------------------------- gloo, several processes
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


ROWS, COLS, LEVELS, ITERS, CHUNK = 104, 45, 2, 8, 3


def _worker(rank, world, port, q, overlap=False, chunk=CHUNK):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [here, os.path.join(root, "oracle"), os.path.join(root, "cpp-optical-flow_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        I0, I1 = synth_pair(1000, ROWS, COLS)
        p = rb.plan(ROWS, COLS, LEVELS, world, 5, chunk)
        comm = rb.DistComm()
        solve = rb.solve_overlapped if overlap else rb.solve
        states = solve([I0], [I1], p, ITERS, [OracleOps(5, 1.0)], comm, [rank])
        u, v = rb.gather_owned(states, p, comm)
        q.put(("ok", rank, None if u is None else (u.copy(), v.copy())))
    except Exception as e:  # pragma: no cover
        q.put(("err", rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,overlap,chunk", [(2, False, CHUNK), (3, False, CHUNK),
                                                 (2, True, CHUNK), (3, True, CHUNK),
                                                 (3, False, (2, 4))])
def test_gloo_bands_equal_undivided_oracle(world, overlap, chunk):
    """Plain and overlapped schedules over torch.distributed point-to-point
    (the code RCCL runs): the posted-then-waited exchange, send copies and
    all, gives the undivided solve's bits."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, overlap, chunk))
             for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
    errs = [r for r in res if r[0] == "err"]
    assert not errs, errs
    (out,) = [r[2] for r in res if r[1] == 0]
    I0, I1 = synth_pair(1000, ROWS, COLS)
    uo, vo = oracle.flow_pyramid(I0, I1, LEVELS, 5, ITERS, 1.0)
    assert np.array_equal(out[0], uo) and np.array_equal(out[1], vo)



# ----------------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def hs():
    import hsflow
    return hsflow


def _bands_on_one_gpu(hs, I0, I1, levels, window, iters, world, chunk, dtype=None,
                      overlap=False, whole=None):
    t0, t1 = torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()
    if dtype is not None:
        t0, t1 = t0.to(dtype), t1.to(dtype)
    rows, cols = I0.shape
    p = rb.plan(rows, cols, levels, world, window, chunk, whole=whole)
    ops = [rb.DeviceOps(window, 1.0, t0.device) for _ in range(world)]
    comm = rb.LocalComm()
    solve = rb.solve_overlapped if overlap else rb.solve
    states = solve([t0] * world, [t1] * world, p, iters, ops, comm, list(range(world)))
    u, v = rb.gather_owned(states, p, comm)
    ref = hs.flow_pyramid_device(t0, t1, levels, window, iters, 1.0)
    torch.cuda.synchronize()
    return (u, v), ref


@pytest.mark.gpu
@pytest.mark.parametrize("world,levels,chunk,window", [(2, 3, 6, 5), (4, 2, 12, 5),
                                                       (3, 3, 8, 3)])
def test_device_bands_bit_identical_to_single_gpu(hs, world, levels, chunk, window):
    I0, I1 = hs.synth_pair(1000, 400, 522)
    (u, v), (ur, vr) = _bands_on_one_gpu(hs, I0, I1, levels, window, 40, world, chunk)
    assert torch.equal(u, ur) and torch.equal(v, vr)


@pytest.mark.gpu
@pytest.mark.parametrize("world,levels,chunk,window", [(2, 3, 6, 5), (3, 2, 8, 3)])
def test_device_overlapped_bands_bit_identical_to_single_gpu(hs, world, levels, chunk, window):
    """The overlapped schedule on the GPU: interiors on each rank's side
    stream, strips on the caller's stream, in-process exchange."""
    I0, I1 = hs.synth_pair(1000, 400, 522)
    (u, v), (ur, vr) = _bands_on_one_gpu(hs, I0, I1, levels, window, 40, world, chunk,
                                         overlap=True)
    assert torch.equal(u, ur) and torch.equal(v, vr)


def _device_gloo_worker(rank, world, port, q, shape, levels, iters, chunk, whole_px=0):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [here, os.path.join(root, "cpp-optical-flow_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import hsflow
        rows, cols = shape
        I0, I1 = hsflow.synth_pair(1000, rows, cols)
        t0 = torch.from_numpy(I0).cuda().half()
        t1 = torch.from_numpy(I1).cuda().half()
        p, _ = rb.fit_plan(rows, cols, levels, world, 5, chunk,
                           whole=rb.whole_levels(rows, cols, levels, world, whole_px))
        comm = rb.DistComm()
        states = rb.solve([t0], [t1], p, iters, [rb.DeviceOps(5, 1.0, t0.device)], comm, [rank])
        u, v = rb.gather_owned(states, p, comm)
        torch.cuda.synchronize()
        if rank == 0:
            ur, vr = hsflow.flow_pyramid_device(t0, t1, levels, 5, iters, 1.0)
            torch.cuda.synchronize()
            nan = int(torch.isnan(u).sum() + torch.isnan(v).sum())
            diff = int((u != ur).sum() + (v != vr).sum())
            q.put(("ok", rank, (nan, diff)))
        else:
            q.put(("ok", rank, None))
    except Exception as e:  # pragma: no cover
        q.put(("err", rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("shape,levels,iters,chunk,whole_px", [
    ((540, 960), 3, 200, (24, 48), 0), ((1080, 1920), 3, 100, (24, 48), 0),
    ((1080, 1920), 3, 100, (24, 48), 600_000)])
def test_device_bands_over_gloo_two_processes(shape, levels, iters, chunk, whole_px):
    """bench.py's bands leg path at N = 2: two processes, DistComm over gloo
    with CUDA tensors (the 2-rank rehearsal's transport; RCCL on a
    multi-GPU node), DeviceOps on the one GPU; rank 0's gathered (u, v)
    equal the single-GPU pyramid solve bit for bit."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_device_gloo_worker,
                         args=(r, world, port, q, shape, levels, iters, chunk, whole_px))
             for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
    errs = [r for r in res if r[0] == "err"]
    assert not errs, errs
    (nan_diff,) = [r[2] for r in res if r[1] == 0]
    assert nan_diff == (0, 0), nan_diff


@pytest.mark.gpu
def test_device_overlapped_bands_8k_fp16_eight_ranks(hs):
    I0, I1 = hs.synth_pair(1000, 4320, 7680)
    (u, v), (ur, vr) = _bands_on_one_gpu(hs, I0, I1, 3, 5, 30, 8, 12, torch.float16,
                                         overlap=True)
    assert torch.equal(u, ur) and torch.equal(v, vr)


@pytest.mark.gpu
@pytest.mark.parametrize("overlap", [False, True])
def test_device_bands_8k_fp16_eight_ranks_whole_coarse_level(hs, overlap):
    """bench.py's bands plan at N = 8: level 2 (1920 x 1080) solved whole on
    every rank, levels 1 and 0 banded -- bit-identical to one GPU."""
    I0, I1 = hs.synth_pair(1000, 4320, 7680)
    whole = rb.whole_levels(4320, 7680, 3, 8, 2_200_000)
    assert whole == (False, False, True)
    (u, v), (ur, vr) = _bands_on_one_gpu(hs, I0, I1, 3, 5, 30, 8, 12, torch.float16,
                                         overlap=overlap, whole=whole)
    assert torch.equal(u, ur) and torch.equal(v, vr)


@pytest.mark.gpu
def test_device_bands_8k_fp16_eight_ranks(hs):
    """Config 5 geometry: 7680x4320 fp16, 3 levels, 8 bands, chunk 12."""
    I0, I1 = hs.synth_pair(1000, 4320, 7680)
    (u, v), (ur, vr) = _bands_on_one_gpu(hs, I0, I1, 3, 5, 30, 8, 12, torch.float16)
    assert torch.equal(u, ur) and torch.equal(v, vr)


@pytest.mark.gpu
@pytest.mark.parametrize("overlap", [False, True])
def test_device_bands_graphed_bit_identical(hs, overlap):
    """row_bands.graphed: the whole banded solve of virtual ranks captured
    into one hipGraph; replays (over NaN-filled outputs) give the undivided
    solve's bits."""
    I0, I1 = hs.synth_pair(1000, 400, 522)
    t0, t1 = torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()
    p = rb.plan(400, 522, 2, 3, 5, 6)
    ops = [rb.DeviceOps(5, 1.0, t0.device) for _ in range(3)]
    solver = rb.solve_overlapped if overlap else rb.solve
    g, u, v = rb.graphed(solver, [t0] * 3, [t1] * 3, p, 40, ops, rb.LocalComm(), [0, 1, 2])
    u.fill_(float("nan"))
    v.fill_(float("nan"))
    g.replay()
    g.replay()
    ur, vr = hs.flow_pyramid_device(t0, t1, 2, 5, 40, 1.0)
    torch.cuda.synchronize()
    assert torch.equal(u, ur) and torch.equal(v, vr)


def test_graphed_refuses_dist_comm():
    p = rb.plan(64, 30, 1, 2, 5, 2)

    class O:
        stream = object()
        device = "cpu"
    with pytest.raises(ValueError):
        rb.graphed(rb.solve, [None] * 2, [None] * 2, p, 4, [O(), O()], rb.DistComm(), [0, 1])


@pytest.mark.gpu
@pytest.mark.parametrize("overlap", [False, True])
def test_device_bands_graphed_with_rank_streams(hs, overlap):
    """The capture round 3 fenced off: every virtual rank on a stream of its
    own.  graphed() forks the rank streams from the capturing stream and,
    while capturing, keeps each rank's work on its rank stream (a stream
    forked from a non-origin capturing stream crashes hipStreamEndCapture on
    ROCm 7.2: scripts/lab/capture_ops.py side2); the whole schedule is
    captured and replays give the undivided solve's bits."""
    I0, I1 = hs.synth_pair(1000, 400, 522)
    t0, t1 = torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()
    p = rb.plan(400, 522, 2, 3, 5, 6)
    ops = [rb.DeviceOps(5, 1.0, t0.device, stream=torch.cuda.Stream()) for _ in range(3)]
    solver = rb.solve_overlapped if overlap else rb.solve
    g, u, v = rb.graphed(solver, [t0] * 3, [t1] * 3, p, 40, ops, rb.LocalComm(), [0, 1, 2])
    u.fill_(float("nan"))
    v.fill_(float("nan"))
    g.replay()
    g.replay()
    ur, vr = hs.flow_pyramid_device(t0, t1, 2, 5, 40, 1.0)
    torch.cuda.synchronize()
    assert torch.equal(u, ur) and torch.equal(v, vr)
