"""Where does the fresh-output cost of hsflow_flow go?  The reference's own
call (main.cpp:93 `cv::Mat u, v;` then :98) at 1080p and 4K, f64 outputs,
median of N calls per variant, alternated:

  reused     np.empty planes reused across calls (cv::Mat::create steady state)
  fresh      new private anonymous pages per call (bench.py's fresh case)
  touched    new pages, every page written by this script before the call
  huge       new pages advised MADV_HUGEPAGE and written before the call

    python scripts/pcie/fresh_probe.py [--reps 9]
"""
import argparse
import json
import mmap
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import hsflow  # noqa: E402


def fresh_planes(rows, cols, mode):
    m = mmap.mmap(-1, 2 * rows * cols * 8, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    if mode == "huge":
        m.madvise(mmap.MADV_HUGEPAGE)
    a = np.frombuffer(m, np.float64).reshape(2, rows, cols)
    if mode in ("touched", "huge"):
        a[:, :, ::512] = 0.0  # one write per 4 KB page
    return m, a


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=9)
    a = ap.parse_args()
    out = {}
    for name, rows, cols, iters in (("1080p", 1080, 1920, 300), ("4k", 2160, 3840, 500)):
        I0, I1 = hsflow.synth_pair(1000, rows, cols, dtype=np.uint8)
        hs = hsflow.hornSchunck(5, iters, 1.0)
        u = np.empty((rows, cols), np.float64)
        v = np.empty((rows, cols), np.float64)
        hs.getFlow(I0, I1, u, v)
        ref = (u.copy(), v.copy())
        ts = {k: [] for k in ("reused", "fresh", "touched", "huge")}
        for _ in range(a.reps):
            for mode in ts:
                if mode == "reused":
                    t = time.perf_counter()
                    hs.getFlow(I0, I1, u, v)
                    ts[mode].append(time.perf_counter() - t)
                    continue
                m, p = fresh_planes(rows, cols, mode)
                t = time.perf_counter()
                hs.getFlow(I0, I1, p[0], p[1])
                ts[mode].append(time.perf_counter() - t)
                ok = np.array_equal(p[0], ref[0]) and np.array_equal(p[1], ref[1])
                del p
                m.close()
                assert ok, mode
        rec = {k: round(sorted(x)[len(x) // 2] * 1e3, 3) for k, x in ts.items()}
        rec["min"] = {k: round(min(x) * 1e3, 3) for k, x in ts.items()}
        out[name] = rec
        print(name, json.dumps(rec), flush=True)
    print("RESULT", json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
