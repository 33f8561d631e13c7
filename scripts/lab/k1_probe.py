"""K1 alone and the solve with / without the batch split, per library build
(same-box A/B; each build in its own process, alternated):
    python scripts/lab/k1_probe.py prev cur"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "cpp-optical-flow_amd")
CHILD = r'''
import sys, time, json
sys.path.insert(0, %(pkg)r)
import hsflow
hsflow.LIB_PATH = %(lib)r
import numpy as np, torch
out = {}
batch, rows, cols, iters = 8, 1080, 1920, 300
ps = [hsflow.synth_pair(1000 + i, rows, cols) for i in range(batch)]
I0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
I1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
ws = hsflow.alloc_workspace(rows, cols, batch)
u = torch.empty((batch, rows, cols), dtype=torch.float32, device="cuda"); v = torch.empty_like(u)
def timed(fn, n=50):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n
out["k1_us"] = round(timed(lambda: hsflow.gradients_device(I0, I1, ws)) * 1e3, 2)
I0u, I1u = I0.to(torch.uint8), I1.to(torch.uint8)
out["k1_u8_us"] = round(timed(lambda: hsflow.gradients_device(I0u, I1u, ws)) * 1e3, 2)
for ms in (1, 2):
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws, s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with hsflow.max_streams_as(ms), torch.cuda.graph(g, capture_error_mode="thread_local"):
        hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws, torch.cuda.current_stream())
    t = time.perf_counter(); n = 0
    while time.perf_counter() - t < 0.15:
        g.replay(); n += 1
        if n %% 4 == 0: torch.cuda.synchronize()
    out[f"solve_ms_streams{ms}"] = round(timed(g.replay, 20), 4)
print("RESULT " + json.dumps(out), flush=True)
'''


def main(names):
    order = (list(names) + list(reversed(names))) * 2
    for n in order:
        lib = os.path.join(PKG, "lab", f"libhsflow_{n}.so")
        r = subprocess.run([sys.executable, "-c", CHILD % {"pkg": PKG, "lib": lib}],
                           capture_output=True, text=True, timeout=240)
        line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")]
        if r.returncode != 0 or not line:
            print(n, "FAILED", r.returncode, r.stderr[-2000:], flush=True)
            return 1
        print(n, line[0][7:], flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
