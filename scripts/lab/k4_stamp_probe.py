"""Per-wave timeline of one K4 launch (lab build `stamp` of
scripts/lab/k4_variants.py): start, duration and placement of every wave
of the last K4 pass of a solve, summarised by how many waves shared the
wave's SIMD and by segment class.

    python scripts/lab/k4_stamp_probe.py [4k1|4k2|1080p8|1440p1] ...   (GPU box)
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

hsflow.LIB_PATH = os.path.join(PKG, "lab", "libhsflow_stamp.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402

SHAPES = {"1080p8": (8, 1080, 1920, 300), "4k2": (2, 2160, 3840, 500),
          "4k1": (1, 2160, 3840, 500), "1080p1": (1, 1080, 1920, 300),
          "1440p1": (1, 1440, 2560, 300)}


def q(a, f):
    return float(np.quantile(a, f))


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
    buf = (ctypes.c_ulonglong * (4 * n))()
    L.hsflow_lab_k4_stamps.restype = ctypes.c_int
    assert L.hsflow_lab_k4_stamps(ctypes.byref(buf), n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 4)
    a = a[a[:, 1] > 0]
    t0 = a[:, 0].min()
    st = (a[:, 0] - t0).astype(np.float64) / 100.0  # us
    en = (a[:, 1] - t0).astype(np.float64) / 100.0
    dur = en - st
    hw = a[:, 2] & 0xFFFFFFFF
    xcc = (a[:, 2] >> 32) & 0xF
    simd_key = (xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 7) | \
        (((hw >> 8) & 15) << 2) | ((hw >> 4) & 3)
    seg = (a[:, 3] >> 32).astype(np.int64)
    # waves whose lifetime overlaps another wave's on the same SIMD
    shared = np.zeros(len(a), dtype=np.int64)
    order = np.argsort(simd_key, kind="stable")
    keys = simd_key[order]
    i = 0
    while i < len(order):
        j = i
        while j < len(order) and keys[j] == keys[i]:
            j += 1
        idx = order[i:j]
        for x in idx:
            shared[x] = sum(1 for y in idx if y != x and st[y] < en[x] and st[x] < en[y])
        i = j
    nseg = int(seg.max()) + 1
    edge = (seg == 0) | (seg == nseg - 1)
    out = {"shape": tag, "waves": int(len(a)), "span_us": round(float(en.max()), 2),
           "start_spread_us": [round(q(st, 0.5), 2), round(q(st, 0.99), 2), round(float(st.max()), 2)],
           "dur_us": {"min": round(float(dur.min()), 2), "median": round(q(dur, 0.5), 2),
                      "p90": round(q(dur, 0.9), 2), "max": round(float(dur.max()), 2)},
           "simds": int(len(np.unique(simd_key)))}
    for k in sorted(set(shared.tolist())):
        m = shared == k
        out[f"shared{k}"] = {"waves": int(m.sum()), "median_us": round(q(dur[m], 0.5), 2),
                             "max_us": round(float(dur[m].max()), 2)}
    out["edge_segments"] = {"waves": int(edge.sum()), "median_us": round(q(dur[edge], 0.5), 2)}
    out["inner_segments"] = {"waves": int((~edge).sum()), "median_us": round(q(dur[~edge], 0.5), 2)}
    late = en > q(en, 0.95)
    out["last5pct"] = {"shared_mean": round(float(shared[late].mean()), 2),
                       "edge_frac": round(float(edge[late].mean()), 2),
                       "start_median_us": round(q(st[late], 0.5), 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    for t in sys.argv[1:] or ["4k1"]:
        run(t)
