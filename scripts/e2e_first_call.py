"""Why is the first bench.e2e_leg call of a process ~12 % slower than later
ones (profiles/r04_e2e_slots_ab.jsonl)?  One mode per process:
    base     e2e_leg twice
    pinned   cycle pinned host buffers of the leg's sizes through torch's
             caching host allocator first, then e2e_leg twice
    device   the same for device buffers (caching device allocator)
    both     both"""
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cpp-optical-flow_amd")]
import torch  # noqa: E402
import bench  # noqa: E402

mode = sys.argv[1]
dev = torch.device("cuda", 0)
shp = (8, 1080, 1920)
if mode in ("pinned", "both"):
    bufs = [torch.empty(shp, dtype=torch.float32).pin_memory() for _ in range(6)] + \
        [torch.empty(shp, dtype=torch.uint8).pin_memory() for _ in range(4)]
    del bufs
if mode in ("device", "both"):
    bufs = [torch.empty(shp, dtype=torch.float32, device=dev) for _ in range(6)] + \
        [torch.empty(shp, dtype=torch.uint8, device=dev) for _ in range(6)]
    del bufs
torch.cuda.synchronize()
args = types.SimpleNamespace(iters=0, window=5, alpha=1.0, no_graph=False)
for i in range(2):
    r = bench.e2e_leg("1080p", args, dev)
    print(json.dumps({"mode": mode, "call": i, "pairs_per_s": r["pairs_per_s_e2e"],
                      "ms_per_batch": r["e2e"]["ms_per_batch"]}), flush=True)
