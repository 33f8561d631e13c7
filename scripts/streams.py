"""Does splitting a batch over S concurrent streams overlap the load and
compute phases of K2?  Times iters Jacobi iterations on B 1080p pairs as
S independent sub-batches on S torch streams (one process, interleaved)."""
import argparse, json, os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "cpp-optical-flow_amd")]
import numpy as np, torch, hsflow
ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=8); ap.add_argument("--iters", type=int, default=40)
ap.add_argument("--streams", default="1,2,4"); ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--rows", type=int, default=1080); ap.add_argument("--cols", type=int, default=1920)
a = ap.parse_args()
R, C, B = a.rows, a.cols, a.batch
pairs = [hsflow.synth_pair(1000 + i, R, C) for i in range(B)]
I0 = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
I1 = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
u = torch.empty_like(I0); v = torch.empty_like(I0)
res = {}
setups = {}
for S in [int(x) for x in a.streams.split(",")]:
    per = B // S
    ss = [torch.cuda.Stream() for _ in range(S)]
    wss = [hsflow.alloc_workspace(R, C, per) for _ in range(S)]
    for k in range(S):
        hsflow.gradients_device(I0[k*per:(k+1)*per], I1[k*per:(k+1)*per], wss[k], stream=ss[k])
    setups[S] = (per, ss, wss)
torch.cuda.synchronize()
for rnd in range(a.rounds):
    for S, (per, ss, wss) in setups.items():
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        cur = torch.cuda.current_stream()
        e0.record(cur)
        for k in range(S):
            ss[k].wait_event(e0)
            hsflow.jacobi_device(R, C, per, 5, a.iters, 1.0, u[k*per:(k+1)*per], v[k*per:(k+1)*per], wss[k], stream=ss[k])
        for k in range(S):
            cur.wait_stream(ss[k])
        e1.record(cur); torch.cuda.synchronize()
        res.setdefault(S, []).append(e0.elapsed_time(e1))
for S, ts in res.items():
    med = float(np.median(ts))
    print(json.dumps({"streams": S, "batch": B, "ms_median": round(med, 4), "Mpix_iter_per_s": round(B * R * C * a.iters / (med * 1e-3) / 1e6, 1)}))
