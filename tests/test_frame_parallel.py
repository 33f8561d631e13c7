"""Multi-process (world_size 2, gloo, CPU) tests of the frame-parallel
driver: scatter -> solve -> gather returns every pair's flow in stream order,
identical to solving the stream on one rank.  The per-pair solver here is the
CPU oracle (test infrastructure); on the GPU the same protocol runs over RCCL
with hsflow.flow_device (bench.py --mode stream)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import frame_parallel as fp
from synth_ref import synth_pair

ROWS, COLS, N_PAIRS = 24, 40, 7


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _solve(I0, I1):
    import oracle
    u, v = oracle.flow(I0.numpy(), I1.numpy(), 5, 6, 1.0)
    return torch.from_numpy(u.astype(np.float32)), torch.from_numpy(v.astype(np.float32))


def _stream():
    return [tuple(torch.from_numpy(a) for a in synth_pair(1000 + j, ROWS, COLS))
            for j in range(N_PAIRS)]


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [here, os.path.join(root, "oracle"), os.path.join(root, "cpp-optical-flow_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        stream = _stream() if rank == 0 else None
        mine = fp.my_pairs(N_PAIRS, rank, world)
        out = fp.run_stream(stream, N_PAIRS, (ROWS, COLS), torch.float32, _solve,
                            torch.device("cpu"), rank, world)
        t = fp.max_over_ranks(0.5 + rank, torch.device("cpu"), world)
        if rank == 0:
            q.put(("ok", [(u.numpy(), v.numpy()) for (u, v) in out], t, mine))
        else:
            q.put(("peer", None, t, mine))
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e), None, None))
    finally:
        dist.destroy_process_group()


def test_ownership_round_robin():
    assert fp.my_pairs(7, 0, 2) == [0, 2, 4, 6]
    assert fp.my_pairs(7, 1, 2) == [1, 3, 5]
    assert sorted(sum((fp.my_pairs(64, r, 8) for r in range(8)), [])) == list(range(64))


def test_scatter_solve_gather_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] != "err" for r in res), res
    ok = [r for r in res if r[0] == "ok"][0]
    flows = ok[1]
    assert len(flows) == N_PAIRS
    assert all(r[2] == 1.5 for r in res)  # max over ranks
    for j, (I0, I1) in enumerate(_stream()):
        u, v = _solve(I0, I1)
        assert np.array_equal(flows[j][0], u.numpy()) and np.array_equal(flows[j][1], v.numpy())


def test_single_rank_path():
    stream = _stream()
    out = fp.run_stream(stream, N_PAIRS, (ROWS, COLS), torch.float32, _solve,
                        torch.device("cpu"), 0, 1)
    assert len(out) == N_PAIRS


def _solve_batch(I0, I1):
    us, vs = zip(*[_solve(a, b) for a, b in zip(I0, I1)])
    return torch.stack(us), torch.stack(vs)


def _uneven_sizes(share):
    """Explicit group sizes, different per share (the bench's are modelled)."""
    return [share] if share < 2 else [share - 1, 1]


def _pipe_worker(rank, world, port, chunks, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [here, os.path.join(root, "oracle"), os.path.join(root, "cpp-optical-flow_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        stream = _stream() if rank == 0 else None
        sizes = _uneven_sizes if chunks == "sizes" else None
        out = fp.run_stream_pipelined(stream, N_PAIRS, (ROWS, COLS), torch.float32,
                                      _solve_batch, torch.device("cpu"), rank, world,
                                      chunks=chunks if sizes is None else 2, sizes=sizes)
        q.put(("ok", [(u.numpy(), v.numpy()) for (u, v) in out]) if rank == 0
              else ("peer", out))
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e)))
    finally:
        dist.destroy_process_group()


def test_chunk_split():
    assert fp.chunk_split([0, 2, 4, 6], 2) == [[0, 2], [4, 6]]
    assert fp.chunk_split([1, 3, 5], 2) == [[1, 3], [5]]
    assert fp.chunk_split([1], 3) == [[1]]
    assert fp.chunk_split([], 2) == []
    assert sum(fp.chunk_split(list(range(9)), 4), []) == list(range(9))


@pytest.mark.parametrize("world,chunks", [(2, 2), (3, 2), (2, 3), (3, 1), (2, "sizes"),
                                          (3, "sizes")])
def test_pipelined_stream_bit_identical(world, chunks):
    """The overlapped schedule (scatter of every group posted up front, group
    c+1 solved while group c's flows travel back) returns every pair's flow
    in stream order, equal to the per-pair solve, for uneven shares (7 pairs
    over 2 and 3 ranks) and any group count."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, chunks, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] != "err" for r in res), res
    assert all(r[1] is None for r in res if r[0] == "peer")
    flows = [r for r in res if r[0] == "ok"][0][1]
    assert len(flows) == N_PAIRS
    for j, (I0, I1) in enumerate(_stream()):
        u, v = _solve(I0, I1)
        assert np.array_equal(flows[j][0], u.numpy()) and np.array_equal(flows[j][1], v.numpy())


def test_group_sizes_model():
    """frame_parallel.group_sizes: one rank takes batches of <= 8; several
    ranks take the non-increasing sizes the pipeline model rates best -- never
    worse than even groups, and a pipeline never beats its solves alone."""
    assert fp.group_sizes(64, 1, 4.1, 16.6) == [8] * 8
    assert fp.group_sizes(5, 1, 4.1, 16.6) == [5]
    assert fp.group_sizes(0, 4, 4.1, 16.6) == []
    for share in (1, 3, 8, 16, 32):
        s = fp.group_sizes(share, 8, 4.1, 16.6)
        assert sum(s) == share and all(0 < g <= 8 for g in s)
        assert list(s) == sorted(s, reverse=True)
        t = fp.pipeline_ms(s, 4.1, 16.6)
        for k in (1, 2, 4):
            even = [share // k + (1 if c < share % k else 0) for c in range(k) if share // k or c < share % k]
            if all(0 < g <= 8 for g in even):
                assert t <= fp.pipeline_ms(even, 4.1, 16.6) + 1e-9
        assert t >= sum(fp.GROUP_SOLVE_MS[g - 1] for g in s) - 1e-9
    # u8 frames move a quarter of f32's bytes: the model never gets slower
    assert fp.pipeline_ms([5, 2, 1], 4.1, 16.6) < fp.pipeline_ms([5, 2, 1], 16.6, 16.6)


@pytest.mark.parametrize("gbps", [25.0, 50.0, 100.0, 150.0])
def test_group_sizes_follow_the_measured_link(gbps):
    """bench.stream_leg sizes the groups with the link rate it measured
    (frame_parallel.measure_link_gbps): valid non-increasing partitions at
    any rate, never worse than the sizes picked for another rate, and a
    faster link never makes the modelled pass slower."""
    for share in (8, 16, 32):
        s = fp.group_sizes(share, 8, 4.1, 16.6, link_gbps=gbps)
        assert sum(s) == share and list(s) == sorted(s, reverse=True)
        t = fp.pipeline_ms(s, 4.1, 16.6, link_gbps=gbps)
        for other in (25.0, 50.0, 100.0, 150.0):
            o = fp.group_sizes(share, 8, 4.1, 16.6, link_gbps=other)
            assert t <= fp.pipeline_ms(o, 4.1, 16.6, link_gbps=gbps) + 1e-9
        if gbps < 150.0:
            faster = fp.group_sizes(share, 8, 4.1, 16.6, link_gbps=2 * gbps)
            assert fp.pipeline_ms(faster, 4.1, 16.6, link_gbps=2 * gbps) <= t + 1e-9


def _link_worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(os.path.dirname(here), "cpp-optical-flow_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fp.measure_link_gbps(torch.device("cpu"), rank, world, 1 << 20)))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_measure_link_gbps_world3():
    """Rank 0 times a round trip to each peer; every rank gets the slowest
    peer's rate (broadcast), finite and positive."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_link_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(3))
    for p in procs:
        p.join(timeout=60)
    assert isinstance(res[0], dict), res
    assert len(res[0]["per_peer"]) == 2 and all(x > 0 for x in res[0]["per_peer"])
    assert all(res[r]["link_gbps"] == res[0]["link_gbps"] for r in range(3))
    m = res[0]["measured_gbps"]
    assert abs(m - min(res[0]["per_peer"])) <= 0.01 * m + 0.001
    assert res[0]["link_gbps"] == min(max(m, 1.0), 1000.0)


def test_pipelined_single_rank_groups():
    out = fp.run_stream_pipelined(_stream(), N_PAIRS, (ROWS, COLS), torch.float32,
                                  _solve_batch, torch.device("cpu"), 0, 1, chunks=3)
    for j, (I0, I1) in enumerate(_stream()):
        u, v = _solve(I0, I1)
        assert np.array_equal(out[j][0].numpy(), u.numpy())


def test_batch_of_views_back_to_back_frames():
    """Frames that lie back to back in one buffer batch as a view (no copy);
    anything else is stacked; both equal torch.stack."""
    A = torch.arange(5 * 4 * 6, dtype=torch.float32).reshape(5, 4, 6)
    cpu = torch.device("cpu")
    b = fp.batch_of([A[1], A[2], A[3]], cpu)
    assert b.data_ptr() == A[1].data_ptr() and torch.equal(b, A[1:4])
    for frames in ([A[0], A[2]], [A[3], A[2]], [A[1], A[1].clone()], [A[0, :, :3], A[1, :, :3]]):
        b = fp.batch_of(frames, cpu)
        assert b.untyped_storage().data_ptr() != A.untyped_storage().data_ptr()  # a copy
        assert torch.equal(b, torch.stack(frames))
    # the single-rank pipeline over a back-to-back stream gives the same flows
    S = _stream()
    A0 = torch.stack([p[0] for p in S])
    A1 = torch.stack([p[1] for p in S])
    out = fp.run_stream_pipelined([(A0[j], A1[j]) for j in range(N_PAIRS)], N_PAIRS,
                                  (ROWS, COLS), torch.float32, _solve_batch, cpu, 0, 1,
                                  chunks=2)
    for j, (I0, I1) in enumerate(S):
        u, v = _solve(I0, I1)
        assert np.array_equal(out[j][0].numpy(), u.numpy())


# ---- the same protocol with the real HIP solver (2 processes, one GPU) ----

def _gpu_solve(I0, I1):
    import hsflow
    u, v = hsflow.flow_device(I0.cuda(), I1.cuda(), 5, 30, 1.0)
    torch.cuda.synchronize()
    return u.cpu(), v.cpu()


G_ROWS, G_COLS, G_PAIRS = 96, 258, 5


def _gpu_stream():
    return [tuple(torch.from_numpy(a) for a in synth_pair(2000 + j, G_ROWS, G_COLS))
            for j in range(G_PAIRS)]


def _gpu_worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [here, os.path.join(root, "oracle"), os.path.join(root, "cpp-optical-flow_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # transport over gloo with host tensors (both ranks share the box's one
    # GPU); each rank solves its pairs with libhsflow on cuda:0
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        stream = _gpu_stream() if rank == 0 else None
        out = fp.run_stream(stream, G_PAIRS, (G_ROWS, G_COLS), torch.float32, _gpu_solve,
                            torch.device("cpu"), rank, world)
        q.put(("ok", [(u.numpy(), v.numpy()) for (u, v) in out]) if rank == 0
              else ("peer", None))
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_frame_parallel_gpu_solver_world2_bit_identical():
    """pairs solved on two ranks (each through the C ABI on
    the GPU) and gathered to rank 0 equal a single-rank solve bit for bit."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=110) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    assert all(r[0] != "err" for r in res), res
    flows = [r for r in res if r[0] == "ok"][0][1]
    assert len(flows) == G_PAIRS
    for j, (I0, I1) in enumerate(_gpu_stream()):
        u, v = _gpu_solve(I0, I1)
        assert np.array_equal(flows[j][0], u.numpy()) and np.array_equal(flows[j][1], v.numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_flow_multi_equals_single_context_bits(devices):
    """hsflow_flow_multi (C/C++ callers, one process, pair j on
    devices[j % n], one host thread + context per listed device; the box
    has one GPU, so the same device is listed up to 3 times = concurrent
    contexts) gives every pair exactly the single-context getFlow bits, in
    pair order, u8 and f32 frames, CV_64FC1 and f32 outputs."""
    import hsflow
    rows, cols = 120, 200
    for dtype, out in ((np.uint8, np.float64), (np.float32, np.float32)):
        pairs = [hsflow.synth_pair(2000 + j, rows, cols, dtype=dtype) for j in range(5)]
        got = hsflow.flow_multi(devices, pairs, 5, 40, 1.0, out_dtype=out)
        ctx = hsflow.Context(0)
        try:
            for (a, b), (u, v) in zip(pairs, got):
                ur, vr = ctx.flow(a, b, 5, 40, 1.0, out_dtype=out)
                assert np.array_equal(u, ur) and np.array_equal(v, vr)
        finally:
            ctx.close()


@pytest.mark.gpu
def test_flow_multi_reports_a_bad_device():
    import hsflow
    a, b = hsflow.synth_pair(1, 16, 16)
    with pytest.raises(hsflow.HsflowError) as e:
        hsflow.flow_multi([0, 99], [(a, b), (a, b)], 5, 1, 1.0)
    assert e.value.status == hsflow.HSFLOW_ERR_NODEV
