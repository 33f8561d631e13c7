"""Per-workgroup phase timeline of the K2 workgroup kernel (development
build with -DHSFLOW_DEV_TRACE, scripts/build_dev.sh trace -DHSFLOW_DEV_TRACE).

Each K2 workgroup records, from wave 0: entry, operator set-up done (loads
arrived), iterations done, stores issued (s_memrealtime, 100 MHz) and its
hardware ids.  One eager bench-shaped solve per workload; prints and saves
the phase statistics:
  load   = set-up done - entry     (u, v, gradient loads + operator set-up)
  iter   = iterations done - set-up done
  store  = stores issued - iterations done
and, chip-wide, how many workgroups are in their load phase while others
compute, and per CU how much the two co-resident workgroups' load phases
overlap.

    HSFLOW_LIB=cpp-optical-flow_amd/libhsflow_dev_trace.so HSFLOW_DEV_TRACE_ON=1 \\
        python scripts/k2_trace.py [--streams 2] [--out profiles/r02_k2_trace.json]
"""
import argparse
import collections
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import hsflow  # noqa: E402

WL = {"1080p": (1080, 1920, 300, 8), "4k": (2160, 3840, 500, 2)}


def read(L, cap=1 << 18):
    buf = np.zeros(cap * 6, dtype=np.uint64)
    n = ctypes.c_size_t(0)
    rc = L.hsflow_dev_trace_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(cap),
                                 ctypes.byref(n))
    assert rc == 0
    return buf[: n.value * 6].reshape(-1, 6)


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def analyse(rec):
    t0 = rec[:, 0].astype(np.int64)
    base = t0.min()
    t = (rec[:, :4].astype(np.int64) - base) / 100.0  # us
    hw = rec[:, 4]
    hwid = (hw & 0xFFFFFFFF).astype(np.int64)
    xcc = (hw >> 32).astype(np.int64) & 0xF
    cu = (hwid >> 8) & 0xF
    sh = (hwid >> 12) & 0x1
    se = (hwid >> 13) & 0x7
    key = xcc * 1000 + se * 100 + sh * 16 + cu
    load, it, st = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
    out = {"workgroups": int(len(t)), "span_us": round(float(t[:, 3].max()), 1),
           "cus_seen": int(len(set(key.tolist())))}
    for name, v in (("load_us", load), ("iter_us", it), ("store_us", st),
                    ("life_us", t[:, 3] - t[:, 0])):
        v = v.tolist()
        out[name] = {"p10": round(pct(v, 0.1), 2), "median": round(statistics.median(v), 2),
                     "p90": round(pct(v, 0.9), 2), "mean": round(statistics.mean(v), 2)}
    # chip-wide: sample every 0.5 us, count workgroups loading / iterating
    ts = np.arange(0, t[:, 3].max(), 0.5)
    loading = np.array([int(((t[:, 0] <= x) & (x < t[:, 1])).sum()) for x in ts])
    iterating = np.array([int(((t[:, 1] <= x) & (x < t[:, 2])).sum()) for x in ts])
    busy = loading + iterating > 0
    out["chip"] = {
        "mean_loading": round(float(loading[busy].mean()), 1),
        "mean_iterating": round(float(iterating[busy].mean()), 1),
        "frac_time_iterating_ge_448": round(float((iterating[busy] >= 448).mean()), 3),
        "loading_hist_by_64": np.bincount(np.minimum(loading[busy] // 64, 8)).tolist()}
    # per CU: fraction of a workgroup's load phase during which another
    # workgroup on the same CU was iterating
    by = collections.defaultdict(list)
    for i, k in enumerate(key.tolist()):
        by[k].append(i)
    cov = []
    for k, idx in by.items():
        idx = np.array(idx)
        A, B = t[idx, 0][:, None], t[idx, 1][:, None]
        I1, I2 = t[idx, 1][None, :], t[idx, 2][None, :]
        ov = np.clip(np.minimum(B, I2) - np.maximum(A, I1), 0, None)
        np.fill_diagonal(ov, 0)
        ln = (B - A)[:, 0]
        ok = ln > 0
        cov.extend(np.minimum(1.0, ov.sum(1)[ok] / ln[ok]).tolist())
    out["load_covered_by_coresident_iter"] = round(float(np.mean(cov)), 3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=0, help="0: library default")
    ap.add_argument("--workloads", default="1080p,4k")
    ap.add_argument("--out", default="")
    ap.add_argument("--raw", default="", help="save the raw records (.npz) here")
    a = ap.parse_args()
    L = hsflow.lib()
    if a.streams:
        hsflow.set_max_streams(a.streams)
    res = {"streams": a.streams or "default"}
    for name in a.workloads.split(","):
        rows, cols, iters, batch = WL[name]
        ps = [hsflow.synth_pair(1000 + i, rows, cols) for i in range(batch)]
        I0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
        I1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
        u, v = torch.empty_like(I0), torch.empty_like(I0)
        ws = hsflow.alloc_workspace(rows, cols, batch)
        for _ in range(2):
            hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws)
        torch.cuda.synchronize()
        read(L)
        hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws)
        torch.cuda.synchronize()
        rec = read(L)
        if a.raw:
            np.savez_compressed(f"{a.raw}_{name}.npz", rec=rec)
        # one pass (the middle launch pair) and the whole solve
        res[name] = {"solve": analyse(rec)}
        print(name, json.dumps(res[name]), flush=True)
        del I0, I1, u, v, ws
        torch.cuda.empty_cache()
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
