"""numpy restatement of hsflow_synth_pair (csrc/hsflow_host.cpp) -- checks the
C generator bit-for-bit so bench inputs are reproducible from Python."""
import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(z):
    z = np.asarray(z, np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def texture(seed, r0, r1, c0, c1):
    R = 3
    rr = np.arange(r0 - R, r1 + R, dtype=np.int64)
    cc = np.arange(c0 - R, c1 + R, dtype=np.int64)
    key = ((rr.astype(np.uint32).astype(np.uint64) << np.uint64(32))[:, None]
           | cc.astype(np.uint32).astype(np.uint64)[None, :])
    n = (splitmix64(splitmix64(np.uint64(seed)) ^ key) >> np.uint64(56)).astype(np.int64)
    cs = np.cumsum(np.pad(n, ((0, 0), (1, 0))), axis=1)
    h = cs[:, 7:] - cs[:, :-7]
    cs = np.cumsum(np.pad(h, ((1, 0), (0, 0))), axis=0)
    S = cs[7:, :] - cs[:-7, :]
    return np.clip(128 + np.floor_divide((S - 6248) * 5, 64), 0, 255)


def synth_pair(seed, rows, cols, qdy=-3, qdx=6):
    qy, qx = -qdy, -qdx
    ty0 = min(0, qy // 4)
    ty1 = max(rows, (4 * (rows - 1) + qy) // 4 + 2)
    tx0 = min(0, qx // 4)
    tx1 = max(cols, (4 * (cols - 1) + qx) // 4 + 2)
    T = texture(seed, ty0, ty1, tx0, tx1)
    I0 = T[-ty0:-ty0 + rows, -tx0:-tx0 + cols]
    y4 = 4 * np.arange(rows) + qy
    x4 = 4 * np.arange(cols) + qx
    y0, fy = y4 // 4, y4 % 4
    x0, fx = x4 // 4, x4 % 4
    Y, X = y0[:, None] - ty0, x0[None, :] - tx0
    FY, FX = fy[:, None], fx[None, :]
    num = ((4 - FY) * (4 - FX) * T[Y, X] + (4 - FY) * FX * T[Y, X + 1]
           + FY * (4 - FX) * T[Y + 1, X] + FY * FX * T[Y + 1, X + 1])
    I1 = (num + 8) >> 4
    return I0.astype(np.float32), I1.astype(np.float32)
