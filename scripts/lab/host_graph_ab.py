"""Same-box A/B of hsflow_flow (the getFlow drop-in call: pageable u8
frames in, CV_64FC1 or f32 u, v out, output buffers reused) with the
device solve launched eagerly against replayed from the context's hipGraph
(hsflow_set_host_graphs), alternated in rounds; bits compared:
    python scripts/lab/host_graph_ab.py
Retired experiment: the context-cached solve graph and its
hsflow_set_host_graphs knob were not kept (profiles/r04_host_graph_ab.jsonl,
DESIGN.md "The host-buffer call"), so this needs that build to run."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "cpp-optical-flow_amd"))
import numpy as np  # noqa: E402
import hsflow  # noqa: E402


def med(fn, n):
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return 1e3 * float(np.median(ts))


ctx = hsflow.Context(0)
for rows, cols, iters in ((1080, 1920, 300), (2160, 3840, 500)):
    a, b = (x.astype(np.uint8) for x in hsflow.synth_pair(1000, rows, cols))
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:  # clocks
        ctx.flow(a, b, 5, iters, 1.0)
    for dt in (np.float64, np.float32):
        out = (np.empty((rows, cols), dt), np.empty((rows, cols), dt))
        res = {"shape": f"{cols}x{rows}", "iters": iters, "out": np.dtype(dt).name,
               "eager_ms": [], "graph_ms": []}
        bits = {}
        for r in range(6):
            for on in (False, True):
                hsflow.set_host_graphs(on)
                ms = med(lambda: ctx.flow(a, b, 5, iters, 1.0, out_dtype=dt, out=out), 15)
                res["graph_ms" if on else "eager_ms"].append(round(ms, 4))
                bits[on] = (out[0].copy(), out[1].copy())
        res["eager_median_ms"] = round(float(np.median(res["eager_ms"])), 4)
        res["graph_median_ms"] = round(float(np.median(res["graph_ms"])), 4)
        res["bits_equal"] = bool(np.array_equal(bits[False][0], bits[True][0])
                                 and np.array_equal(bits[False][1], bits[True][1]))
        print(json.dumps(res), flush=True)
hsflow.set_host_graphs(True)
ctx.close()
