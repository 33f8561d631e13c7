"""PCIe copy rates for the end-to-end leg (bench.py e2e_leg): D2H of a
1080p x 8 (u, v) f32 batch (2 x 66 MB) into pinned host memory on one
stream, on two streams, and split into chunks over four; H2D of the u8
frames for reference."""
import json
import time

import torch

n = 8 * 1080 * 1920
dev = torch.device("cuda", 0)
d = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(2)]
h = [torch.empty(n, dtype=torch.float32).pin_memory() for _ in range(2)]
streams = [torch.cuda.Stream(dev) for _ in range(4)]


def d2h(nstreams, chunks):
    parts = []
    for k in range(2):
        step = n // chunks
        for c in range(chunks):
            parts.append((h[k][c * step:(c + 1) * step], d[k][c * step:(c + 1) * step]))
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i, (hh, dd) in enumerate(parts):
        with torch.cuda.stream(streams[i % nstreams]):
            hh.copy_(dd, non_blocking=True)
    torch.cuda.synchronize()
    return 2 * n * 4 / (time.perf_counter() - t) / 1e9


for cfg in ((1, 1), (2, 1), (2, 2), (4, 2), (4, 4), (1, 1), (2, 1)):
    r = [d2h(*cfg) for _ in range(5)]
    print(json.dumps({"d2h_streams": cfg[0], "chunks_per_plane": cfg[1],
                      "GBps_best": round(max(r), 1), "GBps_median": round(sorted(r)[2], 1)}),
          flush=True)
hu = torch.empty(2 * n, dtype=torch.uint8).pin_memory()
du = torch.empty(2 * n, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(5):
    du.copy_(hu, non_blocking=True)
torch.cuda.synchronize()
print(json.dumps({"h2d_u8_GBps": round(5 * 2 * n / (time.perf_counter() - t) / 1e9, 1)}))
