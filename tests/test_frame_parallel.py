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
