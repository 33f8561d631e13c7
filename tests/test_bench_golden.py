"""BASELINE configs at their stated sizes and lengths against the float64
oracle's golden checksums (tests/golden/bench_golden.*, generated offline by
tests/golden/make_bench_golden.py from oracle/ -- the GPU box never runs the
oracle for these):

  configs[1]  1080p x 300 it, the bench's exact solve: batch 8 split over the
              side streams, captured into a hipGraph and replayed
  configs[2]  4K x 500 it, batch 2, same path
  configs[3]  64 x 1080p pairs through the frame-parallel stream protocol
              (one rank, and two ranks over gloo on the box's one GPU): every
              pair bit-identical to its own solve, pair 0 against the golden
  configs[4]  7680 x 4320 fp16, 3-level pyramid, 1000 iterations per level
              (hornSchunck.cpp:56's loop count at every level)

Tolerance: max|du| / max|u_ref| <= 1e-4 on the strided golden sample and
|dSum| / (n max|u_ref|) <= 1e-4 (north_star)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

pytestmark = pytest.mark.gpu


def _graph_solve(hs, I0, I1, window, iters, levels=1):
    rows, cols = I0.shape[-2:]
    batch = I0.shape[0]
    u = torch.empty(I0.shape, dtype=torch.float32, device=I0.device)
    v = torch.empty_like(u)
    if levels > 1:
        ws = torch.empty(hs.pyramid_workspace_bytes(rows, cols, batch, levels),
                         dtype=torch.uint8, device=I0.device)
    else:
        ws = hs.alloc_workspace(rows, cols, batch, I0.device)

    def solve(s):
        if levels > 1:
            hs.flow_pyramid_device(I0, I1, levels, window, iters, 1.0, u, v, ws, s)
        else:
            hs.flow_device(I0, I1, window, iters, 1.0, u, v, ws, s)
    cap = torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cap):
        solve(cap)
    torch.cuda.current_stream().wait_stream(cap)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        solve(torch.cuda.current_stream())
    u.zero_()
    v.zero_()
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    return u, v


@pytest.mark.parametrize("wl,window", [("1080p", 5), ("4k", 5), ("1080p", 3)])
def test_bench_solve_matches_oracle_golden(hs, wl, window):
    w = bench.WORKLOADS[wl]
    rows, cols, iters, batch = w["rows"], w["cols"], w["iters"], w["batch"]
    pairs = [hs.synth_pair(1000 + i, rows, cols) for i in range(batch)]
    I0 = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    I1 = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    u, v = _graph_solve(hs, I0, I1, window, iters)
    golden = bench.golden_entry(rows, cols, iters, window, 1, 1.0)
    res = bench.parity_check(u[0].cpu().numpy(), v[0].cpu().numpy(), golden)
    assert res["ok"], res
    # and pair 1 equals its own single-pair solve bit for bit
    u1, v1 = hs.flow_device(I0[1:2].contiguous(), I1[1:2].contiguous(), window, iters, 1.0)
    assert torch.equal(u1[0], u[1]) and torch.equal(v1[0], v[1])


def test_config5_8k_fp16_pyramid_full_length(hs):
    w = bench.WORKLOADS["8k"]
    rows, cols, iters, levels = w["rows"], w["cols"], w["iters"], w["levels"]
    a, b = hs.synth_pair(1000, rows, cols)
    I0 = torch.from_numpy(a).cuda().half()[None]
    I1 = torch.from_numpy(b).cuda().half()[None]
    u, v = _graph_solve(hs, I0, I1, 5, iters, levels)
    golden = bench.golden_entry(rows, cols, iters, 5, levels, 1.0)
    assert golden is not None
    res = bench.parity_check(u[0].cpu().numpy(), v[0].cpu().numpy(), golden)
    assert res["ok"], res


C4_PAIRS, C4_ROWS, C4_COLS, C4_ITERS = 64, 1080, 1920, 300


def _c4_stream():
    import hsflow
    return [tuple(torch.from_numpy(x) for x in hsflow.synth_pair(1000 + j, C4_ROWS, C4_COLS))
            for j in range(C4_PAIRS)]


def _c4_digest(u, v):
    """Per-pair digest compared bit for bit across runs: float64 sums of the
    f32 planes and a strided sample."""
    u, v = u.cpu().numpy(), v.cpu().numpy()
    return (float(u.astype(np.float64).sum()), float(v.astype(np.float64).sum()),
            u[::37, ::41].copy(), v[::37, ::41].copy())


def test_config4_stream_64_pairs_one_rank(hs):
    import frame_parallel as fp
    stream = [(a.cuda(), b.cuda()) for a, b in _c4_stream()]
    ws = hs.alloc_workspace(C4_ROWS, C4_COLS, C4_PAIRS)

    def solve_batch(I0, I1):
        return hs.flow_device(I0, I1, 5, C4_ITERS, 1.0, workspace=ws)
    pairs = fp.scatter_pairs(stream, C4_PAIRS, (C4_ROWS, C4_COLS), torch.float32,
                             torch.device("cuda"), 0, 1)
    u, v = solve_batch(torch.stack([p[0] for p in pairs]), torch.stack([p[1] for p in pairs]))
    out = fp.gather_flows([(u[k], v[k]) for k in range(C4_PAIRS)], C4_PAIRS,
                          (C4_ROWS, C4_COLS), torch.device("cuda"), 0, 1)
    assert len(out) == C4_PAIRS
    golden = bench.golden_entry(C4_ROWS, C4_COLS, C4_ITERS, 5, 1, 1.0)
    res = bench.parity_check(out[0][0].cpu().numpy(), out[0][1].cpu().numpy(), golden)
    assert res["ok"], res
    for j in (0, 1, 31, 63):
        uj, vj = hs.flow_device(stream[j][0], stream[j][1], 5, C4_ITERS, 1.0)
        assert torch.equal(uj, out[j][0]) and torch.equal(vj, out[j][1]), j


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _c4_worker(rank, world, port, q, pipelined=False):
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, ROOT, os.path.join(ROOT, "cpp-optical-flow_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import frame_parallel as fp
        import hsflow
        stream = _c4_stream() if rank == 0 else None
        mine = fp.my_pairs(C4_PAIRS, rank, world)
        ws = hsflow.alloc_workspace(C4_ROWS, C4_COLS, len(mine), "cuda")
        # transport: gloo with host tensors (both ranks share the one GPU);
        # each rank solves its share (or each group of it) in one batched
        # call on cuda:0
        if pipelined:
            def solve_batch(I0, I1):
                u, v = hsflow.flow_device(I0.cuda(), I1.cuda(), 5, C4_ITERS, 1.0, workspace=ws)
                torch.cuda.synchronize()
                return u.cpu(), v.cpu()
            out = fp.run_stream_pipelined(stream, C4_PAIRS, (C4_ROWS, C4_COLS), torch.float32,
                                          solve_batch, torch.device("cpu"), rank, world,
                                          chunks=2)
        else:
            pairs = fp.scatter_pairs(stream, C4_PAIRS, (C4_ROWS, C4_COLS), torch.float32,
                                     torch.device("cpu"), rank, world)
            u, v = hsflow.flow_device(torch.stack([p[0] for p in pairs]).cuda(),
                                      torch.stack([p[1] for p in pairs]).cuda(), 5, C4_ITERS,
                                      1.0, workspace=ws)
            torch.cuda.synchronize()
            flows = [(u[k].cpu(), v[k].cpu()) for k in range(len(pairs))]
            out = fp.gather_flows(flows, C4_PAIRS, (C4_ROWS, C4_COLS), torch.device("cpu"),
                                  rank, world)
        q.put(("ok", [_c4_digest(a, b) for a, b in out]) if rank == 0 else ("peer", None))
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("pipelined", [False, True])
def test_config4_stream_64_pairs_two_ranks_bit_identical(hs, pipelined):
    """Config 4 over two ranks: the serial schedule (scatter, solve, gather)
    and bench.py's overlapped one (frame_parallel.run_stream_pipelined, two
    groups per rank) both return every pair's single-GPU bits."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c4_worker, args=(r, 2, port, q, pipelined)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=200) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    assert all(r[0] != "err" for r in res), res
    got = [r for r in res if r[0] == "ok"][0][1]
    assert len(got) == C4_PAIRS
    stream = _c4_stream()
    for j in (0, 1, 2, 33, 63):  # owners alternate between the ranks
        u, v = hs.flow_device(stream[j][0].cuda(), stream[j][1].cuda(), 5, C4_ITERS, 1.0)
        ref = _c4_digest(u, v)
        assert got[j][0] == ref[0] and got[j][1] == ref[1], j
        assert np.array_equal(got[j][2], ref[2]) and np.array_equal(got[j][3], ref[3]), j
