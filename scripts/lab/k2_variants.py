"""K2 lab variants: the product hsflow_kernels.hip with textual patches, each
linked with the product's other objects into cpp-optical-flow_amd/lab/
libhsflow_k2<name>.so (not tracked; travels to the GPU box with the tree).

    python scripts/lab/k2_variants.py build NAME [NAME ...]   # here (hipcc)
    python scripts/lab/k2_variants.py probe NAME [NAME ...]   # GPU box

Variants (timing questions about the single-pair K2 launches):
  base      the product source unchanged (the A/B reference build)
  nosetup   the per-launch operator set-up (alpha^2 + Ix^2 + Iy^2, rsq, three
            products per column pair and row) replaced by plain copies of the
            gradients (timing only: wrong results) -- the most a per-solve
            precomputed operator could save per launch
`probe` runs single 1080p and 4K pairs (hipGraph replays after a 0.15 s
pre-warm) with each build in its own process, alternating the order twice,
and prints Mpix*iter/s per build."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "cpp-optical-flow_amd")
LAB = os.path.join(PKG, "lab")
SRC = os.path.join(PKG, "csrc", "hsflow_kernels.hip")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-fno-slp-vectorize"]

PATCHES = {
    "base": [],
    "nosetup": [("                op_setup(a2c, ixe, iye, ite, ixo, iyo, ito, X[r], Y[r], Tr);",
                 "                X[r] = f2v{ixe, ixo}; Y[r] = f2v{iye, iyo}; f2v Tr = f2v{ite, ito};"
                 " (void)a2c;"),
                ("                f2v Tr;\n", ""),
                ("                op_setup(a2c, ixe, iye, ite, ixo, iyo, ito, X[r], Y[r], T[r]);",
                 "                X[r] = f2v{ixe, ixo}; Y[r] = f2v{iye, iyo}; T[r] = f2v{ite, ito};")],
    # timing only (wrong results): every launch runs 2x / 4x its iterations
    # in the same workgroup lifetime (the halo is too shallow for them), so
    # the solve-time difference is the iteration sweep alone -- how much of
    # a single-pair launch the per-launch load / set-up / store / launch gap
    # costs (round 6, the register-resident persistent-kernel question)
    "it2": [("    const int n_it = p.iters;\n    for (int it = 0;",
             "    const int n_it = p.iters * 2;\n    for (int it = 0;"),
            ("    const int n_it = p.iters;\n    // The vertical",
             "    const int n_it = p.iters * 2;\n    // The vertical")],
    "it4": [("    const int n_it = p.iters;\n    for (int it = 0;",
             "    const int n_it = p.iters * 4;\n    for (int it = 0;"),
            ("    const int n_it = p.iters;\n    // The vertical",
             "    const int n_it = p.iters * 4;\n    // The vertical")],
}


def build(name):
    os.makedirs(LAB, exist_ok=True)
    src = open(SRC).read()
    for old, new in PATCHES[name]:
        assert old in src, (name, old)
        src = src.replace(old, new)
    path = os.path.join(PKG, "csrc", f"_lab_kernels_{name}.hip")
    with open(path, "w") as f:
        f.write(src)
    obj = os.path.join(LAB, f"kernels_{name}.o")
    try:
        subprocess.check_call(["/opt/rocm/bin/hipcc", *FLAGS, "-c", path, "-o", obj])
    finally:
        os.remove(path)
    objs = [os.path.join(PKG, "build", f) for f in sorted(os.listdir(os.path.join(PKG, "build")))
            if f.endswith(".o") and f != "hsflow_kernels.o"]
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-shared", "--offload-arch=gfx950", "-o",
                           os.path.join(LAB, f"libhsflow_k2{name}.so"), *objs, obj,
                           "-Wl,-rpath,/opt/rocm/lib"])
    print("built", name, flush=True)


CHILD = r'''
import os, sys, time, json
sys.path.insert(0, %(pkg)r)
import hsflow
hsflow.LIB_PATH = %(lib)r
import numpy as np, torch
out = {}
for tag, batch, rows, cols, iters in (("1080p1", 1, 1080, 1920, 300), ("4k1", 1, 2160, 3840, 500)):
    ps = [hsflow.synth_pair(1000 + i, rows, cols) for i in range(batch)]
    I0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
    I1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
    u = torch.empty((batch, rows, cols), dtype=torch.float32, device="cuda"); v = torch.empty_like(u)
    ws = hsflow.alloc_workspace(rows, cols, batch)
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws, s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with hsflow.max_streams_as(2), torch.cuda.graph(g, capture_error_mode="thread_local"):
        hsflow.flow_device(I0, I1, 5, iters, 1.0, u, v, ws, torch.cuda.current_stream())
    t = time.perf_counter(); n = 0
    while time.perf_counter() - t < 0.15:
        g.replay(); n += 1
        if n %% 4 == 0: torch.cuda.synchronize()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): g.replay()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    out[tag] = {"ms": round(ms, 4), "Mpix_iter_s": round(batch * rows * cols * iters / ms / 1e3),
                "u_sum": float(u.double().sum())}
print("RESULT " + json.dumps(out), flush=True)
'''


def probe(names):
    res = {n: [] for n in names}
    order = list(names) + list(reversed(names))
    for n in order:
        lib = os.path.join(LAB, f"libhsflow_k2{n}.so")
        code = CHILD % {"pkg": PKG, "lib": lib}
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                           timeout=240)
        line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")]
        if r.returncode != 0 or not line:
            print(n, "FAILED", r.returncode, r.stderr[-2000:], flush=True)
            return 1
        res[n].append(json.loads(line[0][7:]))
        print(n, line[0][7:], flush=True)
    print(json.dumps({n: {k: max(x[k]["Mpix_iter_s"] for x in v) for k in v[0]}
                      for n, v in res.items()}), flush=True)
    return 0


if __name__ == "__main__":
    cmd, names = sys.argv[1], sys.argv[2:]
    if cmd == "build":
        for n in names:
            build(n)
    else:
        sys.exit(probe(names))
