"""Same-box A/B of bench.e2e_leg's device slots (2 = double buffering, 3),
alternated twice.  python scripts/e2e_slots_ab.py"""
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cpp-optical-flow_amd")]
import torch  # noqa: E402
import bench  # noqa: E402

args = types.SimpleNamespace(iters=0, window=5, alpha=1.0, no_graph=False)
dev = torch.device("cuda", 0)
for slots in (2, 3, 2, 3):
    r = bench.e2e_leg("1080p", args, dev, slots=slots)
    print(json.dumps({"slots": slots, "pairs_per_s": r["pairs_per_s_e2e"],
                      "ms_per_batch": r["e2e"]["ms_per_batch"]}), flush=True)
    torch.cuda.empty_cache()
