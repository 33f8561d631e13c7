"""Which part of the overlapped band schedule breaks a hipGraph capture when
every virtual rank has its own stream (tests/test_row_bands.py
::test_device_bands_graphed_with_rank_streams[True] segfaults inside
hipStreamEndCapture; the plain schedule with rank streams captures fine).

    python scripts/lab/capture_bisect.py MODE [LEVELS WORLD ITERS CHUNK]
      nosplit   the library does not split a batch over its side streams
                (hsflow_set_max_streams(1)): the strips solve of every rank
                runs on the rank's stream alone
      noside    the interior solve runs on the rank stream (no per-rank side
                stream), the library still splits the strips batch
      full      the schedule as the test runs it
Each mode in its own process: a crash ends the process."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "cpp-optical-flow_amd")]
import hsflow  # noqa: E402
import row_bands as rb  # noqa: E402


class NoSide(rb.DeviceOps):
    def fork(self):
        pass

    def join(self):
        pass

    def jacobi_stack(self, ws, U, V, n, side=False):
        super().jacobi_stack(ws, U, V, n, side=False)


def main(mode, levels=2, world=3, iters=40, chunk=6):
    I0, I1 = hsflow.synth_pair(1000, 400, 522)
    t0, t1 = torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()
    p = rb.plan(400, 522, levels, world, 5, chunk)
    cls = NoSide if mode == "noside" else rb.DeviceOps
    ops = [cls(5, 1.0, t0.device, stream=torch.cuda.Stream()) for _ in range(world)]
    if mode == "nosplit":
        hsflow.set_max_streams(1)
    print(f"{mode} levels {levels} world {world} iters {iters} chunk {chunk}: capturing",
          flush=True)
    g, u, v = rb.graphed(rb.solve_overlapped, [t0] * world, [t1] * world, p, iters, ops,
                         rb.LocalComm(), list(range(world)))
    u.fill_(float("nan"))
    v.fill_(float("nan"))
    g.replay()
    g.replay()
    ur, vr = hsflow.flow_pyramid_device(t0, t1, levels, 5, iters, 1.0)
    torch.cuda.synchronize()
    ok = bool(torch.equal(u, ur) and torch.equal(v, vr))
    print(f"{mode}: captured, replays bit-identical to the undivided solve: {ok}", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], *[int(x) for x in sys.argv[2:]]))
