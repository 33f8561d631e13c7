"""Minimal reproducer of the round-3 hipStreamEndCapture crash
(row_bands.graphed with a stream per virtual rank).

    python scripts/lab/capture_isolation.py forked     # the fixed order
    python scripts/lab/capture_isolation.py isolated   # round 3's order

During a stream capture (torch.cuda.graph, thread_local mode) a second
stream B issues work:
  forked    B first waits on the capturing stream A (B joins the capture),
            runs its kernel, and A waits on B before the capture ends: the
            work is captured, the graph replays it.  What graphed() does now.
  isolated  B runs its kernel WITHOUT joining the capture (so the kernel runs
            eagerly, uncaptured), then A waits on an event recorded on B.
            CUDA refuses that wait (cudaErrorStreamCaptureIsolation); the
            round-3 solve did exactly this with its rank streams (their first
            operations -- the pyramid build -- came before any wait on the
            capturing stream) and the process crashed inside
            hipStreamEndCapture.
Run each order in its own process (a crash ends it)."""
import sys

import torch


def main(mode):
    dev = torch.device("cuda", 0)
    x = torch.zeros(1 << 20, device=dev)
    y = torch.zeros_like(x)
    A = torch.cuda.Stream(dev)
    B = torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, stream=A, capture_error_mode="thread_local"):
            if mode == "forked":
                B.wait_stream(A)
            with torch.cuda.stream(B):
                x.add_(1.0)
            A.wait_stream(B)
            y.copy_(x)
    except Exception as e:  # the runtime may report the isolation instead
        print(f"{mode}: capture raised {type(e).__name__}: {e}", flush=True)
        return 1
    torch.cuda.synchronize()
    x.zero_()
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    print(f"{mode}: captured; after two replays x = {float(x[0])}, y = {float(y[0])} "
          f"(the captured add runs per replay: 2.0 / 2.0 if B joined the capture)", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "forked"))
