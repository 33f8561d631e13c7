"""Which torch operation on a second (forked) stream breaks hipStreamEndCapture
(the overlapped band schedule with rank streams segfaults there, the plain
one does not; scripts/lab/capture_bisect.py).  One operation per process:

    python scripts/lab/capture_ops.py MODE
      alloc    torch.zeros / torch.empty on the forked stream
      stack    torch.stack of row views on the forked stream
      foreach  torch._foreach_copy_ of row views on the forked stream
      foreach_origin  the same copies on the capture's origin stream
      side2    a third stream forked from the second and joined back: CRASHES
               inside hipStreamEndCapture (a stream whose first capture
               dependency is a non-origin capturing stream)
      side2_pre  the same, with the third stream first forked from the origin
The capture forks stream B from the origin A, runs MODE's work on B, joins
B back into A and ends the capture; then replays once and checks values."""
import sys

import torch


def main(mode):
    dev = torch.device("cuda", 0)
    base = torch.arange(64 * 32, dtype=torch.float32, device=dev).reshape(64, 32)
    out = torch.zeros(2, 8, 32, device=dev)
    A, B, C = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=A, capture_error_mode="thread_local"):
        if mode == "side2_pre":
            C.wait_stream(A)  # C joins the capture through the origin first
        B.wait_stream(A)
        with torch.cuda.stream(B):
            if mode == "alloc":
                z = torch.zeros(8, 32, device=dev)
                out[0].copy_(z + base[0:8])
            elif mode == "stack":
                s = torch.stack([base[0:8], base[8:16]])
                out.copy_(s)
            elif mode == "foreach":
                torch._foreach_copy_([out[0], out[1]], [base[0:8], base[8:16]])
            elif mode in ("side2", "side2_pre"):
                C.wait_stream(B)
                with torch.cuda.stream(C):
                    out[0].copy_(base[0:8])
                B.wait_stream(C)
        if mode == "foreach_origin":
            A.wait_stream(B)
            torch._foreach_copy_([out[0], out[1]], [base[0:8], base[8:16]])
        A.wait_stream(B)
    torch.cuda.synchronize()
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    print(f"{mode}: captured and replayed, out[0,0,:3] = {out[0, 0, :3].tolist()}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
