"""bench.py's N > 1 code path on CPU: world_size 2 over gloo (the driver runs
it over RCCL, one process per GPU).  The timing rule (barrier, K timed steps,
max over ranks) and the config-4 stream leg (rank 0 scatters the pairs,
each rank solves its share in one batched call, rank 0 gathers) run exactly
as in bench.py; only the per-batch solver is injected -- the CPU oracle here,
hsflow.flow_device on the GPU."""
import os
import socket
import sys
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

ROWS, COLS, ITERS, N_PAIRS = 24, 40, 6, 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _solve_batch(I0, I1):
    import oracle
    us, vs = [], []
    for a, b in zip(I0, I1):
        u, v = oracle.flow(a.numpy(), b.numpy(), 5, ITERS, 1.0)
        us.append(torch.from_numpy(u.astype(np.float32)))
        vs.append(torch.from_numpy(v.astype(np.float32)))
    return torch.stack(us), torch.stack(vs)


def _worker(rank, world, port, q):
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, ROOT, os.path.join(ROOT, "oracle"),
                    os.path.join(ROOT, "cpp-optical-flow_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        bench.WORKLOADS["tiny"] = dict(rows=ROWS, cols=COLS, iters=ITERS, batch=2)
        args = types.SimpleNamespace(iters=0, pairs=N_PAIRS, steps=2, window=5, alpha=1.0)
        dev = torch.device("cpu")
        # the timing rule: rank 1 is slower, every rank reports the max
        calls = []
        el = bench.timed_region(lambda: calls.append(1) or (rank and __import__("time").sleep(0.05)),
                                lambda: None, 3, 2, world, dev)
        ref = None
        if rank == 0:
            # the resident leg's input type: f32 frames of the same seeds
            from synth_ref import synth_pair
            ps = [synth_pair(1000 + j, ROWS, COLS) for j in range(N_PAIRS)]
            ref = _solve_batch(torch.from_numpy(np.stack([p[0] for p in ps])),
                               torch.from_numpy(np.stack([p[1] for p in ps])))
        leg = bench.stream_leg("tiny", args, world, rank, dev, solve_batch=_solve_batch,
                               ref=ref)
        q.put((rank, len(calls), el, leg))
    except Exception as e:  # pragma: no cover
        q.put((rank, None, None, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_timing_and_stream_leg_over_gloo(world):
    """The stream leg over gloo: u8 frames scattered from rank 0, each rank's
    share in the modelled group sizes, (u, v) gathered one message per plane
    batch; every gathered pair equals the direct f32 solve bit for bit."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, ncalls, el, leg = q.get(timeout=240)
        res[rank] = (ncalls, el, leg)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert res[r][0] == 5, res[r]  # warmup 2 + timed 3
    # max over ranks: every rank reports the slow ranks' time (>= 3 x 50 ms)
    assert all(res[r][1] == res[0][1] for r in range(world)) and res[0][1] >= 0.15
    leg0, leg1 = res[0][2], res[1][2]
    assert isinstance(leg0, dict), leg0
    assert leg0["gathered"] == N_PAIRS and leg0["finite"] and leg0["transport"] == "gloo (cpu tensors)"
    assert leg0["pairs_per_s"] == leg1["pairs_per_s"] > 0  # max-over-ranks time
    assert leg0["frames"] == "u8" and sum(leg0["group_sizes"]) == len(range(0, N_PAIRS, world))
    assert leg0["parity"]["bitwise_vs_resident"] == {"pairs": N_PAIRS, "identical": N_PAIRS}
    assert leg0["parity"]["ok"]
    # the link was measured before the timed passes (every peer of rank 0)
    # and every rank sized its groups with the same broadcast rate
    assert len(leg0["link_gbps_per_peer"]) == world - 1
    assert all(x > 0 for x in leg0["link_gbps_per_peer"])
    for r in range(world):
        assert res[r][2]["link_gbps_model"] == leg0["link_gbps_model"] > 0


def test_stream_leg_gathers_every_pair_in_order_one_rank():
    """world 1: the same leg without communication returns all pairs."""
    sys.path[:0] = [ROOT]
    import bench
    bench.WORKLOADS["tiny"] = dict(rows=ROWS, cols=COLS, iters=ITERS, batch=2)
    args = types.SimpleNamespace(iters=0, pairs=3, steps=1, window=5, alpha=1.0)
    leg = bench.stream_leg("tiny", args, 1, 0, torch.device("cpu"), solve_batch=_solve_batch)
    assert leg["gathered"] == 3 and leg["finite"] and leg["transport"] == "none (one rank)"


# ------------------------------------------------------- config-5 bands leg
B_ROWS, B_COLS, B_LEVELS, B_ITERS, B_CHUNK = 104, 45, 2, 8, 3


def _bands_worker(rank, world, port, q, overlap, split="auto"):
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, ROOT, os.path.join(ROOT, "oracle"),
                    os.path.join(ROOT, "cpp-optical-flow_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from test_row_bands import OracleOps
        bench.WORKLOADS["tinyb"] = dict(rows=B_ROWS, cols=B_COLS, iters=B_ITERS, batch=1,
                                        levels=B_LEVELS, dtype="f32")
        args = types.SimpleNamespace(workload="tinyb", iters=0, levels=0, dtype=None,
                                     window=5, alpha=1.0, chunk=B_CHUNK, overlap=overlap,
                                     mode="resident", split=split)
        out = []
        leg = bench.bands_leg(args, world, rank, torch.device("cpu"), steps=2, warmup=1,
                              ops=OracleOps(5, 1.0), result=out)
        q.put((rank, leg, out[0] if out else None))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("overlap,split", [(False, "auto"), (False, "rows"), (True, "auto")])
def test_bench_bands_leg_over_gloo(overlap, split):
    """bench.bands_leg -- the default run's configs[4] leg at N > 1 -- with 2
    ranks over gloo: frames broadcast from rank 0, row bands with the halo
    exchange after every chunk (the code RCCL runs), timed with the driver's
    rule, rank 0 gathers; the gathered (u, v) equal the undivided solve bit
    for bit (the CPU oracle is the band solver here, libhsflow on the GPU)."""
    sys.path[:0] = [ROOT]
    import oracle
    from synth_ref import synth_pair
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bands_worker, args=(r, world, port, q, overlap, split))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, leg, uv = q.get(timeout=240)
        res[rank] = (leg, uv)
    for p in procs:
        p.join(timeout=60)
    leg0, leg1 = res[0][0], res[1][0]
    assert isinstance(leg0, dict) and isinstance(leg1, dict), (leg0, leg1)
    assert leg0["n_ranks"] == 2 and leg0["transport"] == "gloo (cpu tensors)"
    # the coarse level (52 x 23 px) is small enough to be solved whole on
    # every rank (bench.BANDS_WHOLE_MAX_PX): exchanges only at level 0
    assert leg0["whole_levels"] == [1]
    # auto: a grid of blocks (2 x 1 for this 104 x 45 frame), rows with --overlap
    assert leg0["split"] == ("blocks 2x1" if split == "auto" and not overlap else "rows")
    assert leg0["exchanges_per_solve"] == -(-B_ITERS // B_CHUNK)
    assert leg0["chunks_per_level"] == [B_CHUNK] * B_LEVELS
    assert leg0["ms_per_pair"] == leg1["ms_per_pair"] > 0  # max over ranks
    assert leg0["parity"]["ok"] is None  # no committed golden at this size
    I0, I1 = synth_pair(1000, B_ROWS, B_COLS)
    uo, vo = oracle.flow_pyramid(I0, I1, B_LEVELS, 5, B_ITERS, 1.0)
    u, v = res[0][1]
    assert np.array_equal(u, uo) and np.array_equal(v, vo)
