"""Per-block timeline of K4 waves (lab build `bstamp` of
scripts/lab/k4_variants.py): shader-clock cycles of each unrolled 12-step
block of a wave's stream (blocks 1-2 are the pipeline fill), median over
the interior segments' waves of the last K4 pass of a solve.

    python scripts/lab/k4_bstamp_probe.py [4k1|4k2|1080p8] ...   (GPU box)
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "cpp-optical-flow_amd")
sys.path.insert(0, PKG)
import hsflow  # noqa: E402

hsflow.LIB_PATH = os.path.join(PKG, "lab", f"libhsflow_{os.environ.get('K4_BSTAMP_LIB', 'bstamp')}.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402

SHAPES = {"1080p8": (8, 1080, 1920, 300), "4k2": (2, 2160, 3840, 500),
          "4k1": (1, 2160, 3840, 500)}


def run(tag):
    batch, rows, cols, iters = SHAPES[tag]
    ps = [hsflow.synth_pair(1000 + i, rows, cols) for i in range(batch)]
    I0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
    I1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
    u = torch.empty((batch, rows, cols), dtype=torch.float32, device="cuda")
    v = torch.empty_like(u)
    ws = hsflow.alloc_workspace(rows, cols, batch)
    s = torch.cuda.current_stream()
    t = time.perf_counter()
    while time.perf_counter() - t < 0.3:
        hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws, s)
    torch.cuda.synchronize()
    L = hsflow.lib()
    n = 16384
    buf = (ctypes.c_ulonglong * (16 * n))()
    assert L.hsflow_lab_k4_bstamps(ctypes.byref(buf), n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 16).astype(np.int64)
    nblk = (a[:, 15] >> 56) & 0xFF
    end = a[:, 15] & ((1 << 56) - 1)
    ok = (nblk > 0) & (a[:, 0] > 0)
    per_block = []
    waves = np.nonzero(ok)[0]
    for w in waves:
        nb = int(nblk[w])
        st = list(a[w, :nb]) + [int(end[w])]
        per_block.append([st[i + 1] - st[i] for i in range(nb)])
    nb_mode = max(set(len(p) for p in per_block), key=[len(p) for p in per_block].count)
    pb = np.array([p for p in per_block if len(p) == nb_mode], dtype=np.float64)
    out = {"shape": tag, "waves": int(len(waves)), "blocks": nb_mode,
           "cycles_per_block_median": [round(float(x)) for x in np.median(pb, axis=0)],
           "cycles_per_step_median": [round(float(x) / 12, 1) for x in np.median(pb, axis=0)],
           "wave_cycles_median": round(float(np.median(pb.sum(axis=1))))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    for t in sys.argv[1:] or ["4k1"]:
        run(t)
