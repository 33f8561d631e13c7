import sys, os
sys.path[:0] = ["cpp-optical-flow_amd", "oracle", "tests"]
import numpy as np
import torch, hsflow, oracle
from conftest import GOLDEN
z = dict(np.load(os.path.join(GOLDEN, "crop64x48.npz")))
I0, I1 = z["I0"], z["I1"]
ctx = hsflow.Context(0)
for kb in (1, 4):
    hsflow.set_iters_per_launch(kb)
    u, v = ctx.flow(I0, I1, 5, 1, 1.0)
    uo, vo = oracle.flow(I0, I1, 5, 1, 1.0)
    bad = np.abs(u - uo) > 1e-4 * np.abs(uo).max()
    print("kb", kb, "bad count", bad.sum(), "rows", np.unique(np.nonzero(bad)[0])[:20], "cols", np.unique(np.nonzero(bad)[1])[:64])
    r, c = np.nonzero(bad)
    for i in range(min(5, len(r))):
        print("  ", r[i], c[i], u[r[i], c[i]], uo[r[i], c[i]])
gx, gy, gt = ctx.gradients(I0, I1)
print("grad ok", np.array_equal(gx, z["gx"]))
# single row
a = np.array([[10, 50, 20, 200, 30, 40, 90]], np.uint8); b = a[:, ::-1].copy()
hsflow.set_iters_per_launch(0)
u, v = ctx.flow(a, b, 5, 1, 1.0); uo, vo = oracle.flow(a, b, 5, 1, 1.0)
print("row u", u, "\noracle", uo)
print(oracle.gradients(a, b))
print(ctx.gradients(a, b))
