"""Generate the committed golden fixtures under tests/golden/.

Run ONCE in the build container (it reads the reference's image files, which
exist only there):  python tests/golden/make_golden.py

What it does
------------
1. Reads the KITTI frames the reference's main.cpp:42-44 uses
   (HornSchunckOF/img/leftimage/0000{40,50}_1{0,1}.png) and converts them to
   gray exactly as main.cpp:13-14 does under OpenCV 4.x (cv::imread gives BGR,
   cvtColor BGR2GRAY = (9798 R + 19235 G + 3735 B + 16384) >> 15).  The gray
   frames are committed as binary PGM (P5): they are the inputs of every
   KITTI parity test, so no test needs /root/reference at run time.
2. Extracts the reference's OWN output -- the arrow plots
   HornSchunckOF/img/resimage/0000{40,50}_10.pnghsbresenhamLineFlow.png
   written by plotFlow.cpp:87 after hs.getFlow(ws=5, 100 it, alpha=1)
   (main.cpp:94-104) -- as label maps: the pixels painted pure green
   (line, plotFlow.cpp:82/86) and pure red (end point, plotFlow.cpp:88).
   These are the reference-produced known-answer test (KAT).
3. Computes float64 golden (u, v) with an INDEPENDENT numpy/scipy
   restatement of hornSchunck.cpp (below; it shares no code with
   oracle/hs_oracle.c) on crops, for several windows/iteration counts, and
   verifies it reproduces the KAT label maps pixel-exactly.

The fixtures are data (inputs and expected outputs); no reference source is
copied.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
from scipy import ndimage

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/HornSchunckOF/img"


# ---------------------------------------------------------------- numpy twin
def gray15(rgb: np.ndarray) -> np.ndarray:
    """main.cpp:13-14 cvtColor(BGR2GRAY), OpenCV 4.x 15-bit fixed point."""
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    return ((9798 * r + 19235 * g + 3735 * b + 16384) >> 15).astype(np.uint8)


def np_gradients(I0, I1):
    """hornSchunck.cpp:19-41 via scipy.ndimage.correlate; mode='mirror' is
    OpenCV's reflect-101 (BORDER_DEFAULT)."""
    a = np.asarray(I0, np.float64)
    b = np.asarray(I1, np.float64)
    sob_x = np.array([[-1, 0, 1], [-2, 0, 2], [-1, 0, 1]], np.float64)
    gx = ndimage.correlate(a, sob_x, mode="mirror")
    gy = ndimage.correlate(a, sob_x.T, mode="mirror")
    return gx, gy, b - a


def np_box(u, w):
    """filter2D(u, ones(w,w)/w^2, anchor (w-w/2-1), BORDER_CONSTANT 0)."""
    a = w - w // 2 - 1
    k = 1.0 / float(w) ** 2
    rows, cols = u.shape
    p = np.zeros((rows + w - 1, cols + w - 1))
    p[a:a + rows, a:a + cols] = u
    s = np.zeros_like(u)
    for i in range(w):
        for j in range(w):
            s = s + k * p[i:i + rows, j:j + cols]
    return s


def np_flow(I0, I1, w, iters, alpha, u0=None, v0=None):
    """hornSchunck.cpp:43-75."""
    gx, gy, gt = np_gradients(I0, I1)
    u = np.zeros_like(gx) if u0 is None else u0.copy()
    v = np.zeros_like(gx) if v0 is None else v0.copy()
    a2 = float(alpha) ** 2
    for _ in range(iters):
        ua, va = np_box(u, w), np_box(v, w)
        c = (gx * ua + gy * va + gt) / (a2 + gx * gx + gy * gy)
        u, v = ua - gx * c, va - gy * c
    return u, v


def py_plot_labels(rows, cols, u, v, delta=20, scale=20.0, outlier=5):
    """plotFlow.cpp:68-88 on a blank canvas -> label map (1 green, 2 red)."""
    lab = np.zeros((rows, cols), np.uint8)
    scale = float(np.float32(scale))

    def setpix(x, y, val):
        if 0 <= x < rows - 1 and 0 <= y < cols - 1:
            lab[x, y] = val

    def sign(x):
        return -1 if x < 0 else (1 if x > 0 else 0)

    def line(x0, y0, x1, y1):
        dX, dY = x1 - x0, y1 - y0
        sX, sY = sign(dX), sign(dY)
        dX, dY = abs(dX), abs(dY)
        dist = max(dX, dY)
        R = float(dist // 2)
        x, y = x0, y0
        for _ in range(dist):
            setpix(x, y, 1)
            if dX > dY:
                x += sX
                R += dY
                if R >= dX:
                    y += sY
                    R -= dX
            else:
                y += sY
                R += dX
                if R >= dY:
                    x += sX
                    R -= dY

    for x1 in range(0, rows, delta):
        for y1 in range(0, cols, delta):
            uu, vv = float(u[x1, y1]), float(v[x1, y1])
            x2 = int(x1 + uu * scale)
            y2 = int(y1 + vv * scale)
            if outlier > 0:
                if -outlier < uu < outlier and -outlier < vv < outlier:
                    line(x1, y1, x2, y2)
            else:
                line(x1, y1, x2, y2)
            setpix(x2, y2, 2)
    return lab


# ------------------------------------------------------------------ helpers
def write_pgm(path, img):
    img = np.ascontiguousarray(img, np.uint8)
    with open(path, "wb") as f:
        f.write(b"P5\n%d %d\n255\n" % (img.shape[1], img.shape[0]))
        f.write(img.tobytes())


def read_png_rgb(path):
    from PIL import Image
    return np.asarray(Image.open(path).convert("RGB"))


def ref_labels(plot_rgb):
    """Reference plot -> label map.  setPixelColor (plotFlow.cpp:24-32) writes
    [0]=r,[1]=g,[2]=b into BGR memory: line (0,255,0) is green, end point
    (0,0,255) in BGR memory is pure red."""
    lab = np.zeros(plot_rgb.shape[:2], np.uint8)
    g = (plot_rgb[..., 0] == 0) & (plot_rgb[..., 1] == 255) & (plot_rgb[..., 2] == 0)
    r = (plot_rgb[..., 0] == 255) & (plot_rgb[..., 1] == 0) & (plot_rgb[..., 2] == 0)
    lab[g] = 1
    lab[r] = 2
    return lab


def main():
    if not os.path.isdir(REF):
        sys.exit("reference images not present; fixtures are already committed")
    meta = {"generator": "tests/golden/make_golden.py", "kat": {}}
    grays = {}
    for tag in ("000050", "000040"):
        prev_rgb = read_png_rgb(f"{REF}/leftimage/{tag}_10.png")
        next_rgb = read_png_rgb(f"{REF}/leftimage/{tag}_11.png")
        raw_prev = read_png_rgb(f"{REF}/resimage/{tag}_10.pngimagePrevRaw.png")
        assert np.array_equal(prev_rgb, raw_prev), "raw copy differs from input"
        g0, g1 = gray15(prev_rgb), gray15(next_rgb)
        grays[tag] = (g0, g1)
        write_pgm(f"{HERE}/kitti_{tag}_10.pgm", g0)
        write_pgm(f"{HERE}/kitti_{tag}_11.pgm", g1)
        plot = read_png_rgb(f"{REF}/resimage/{tag}_10.pnghsbresenhamLineFlow.png")
        lab_ref = ref_labels(plot)
        # raw pixels that are pure green/red by themselves would alias labels
        amb = ref_labels(prev_rgb) != 0
        u, v = np_flow(g0, g1, 5, 100, 1.0)
        lab_np = py_plot_labels(g0.shape[0], g0.shape[1], u, v)
        mism = int(np.count_nonzero((lab_np != lab_ref) & ~amb))
        print(f"{tag}: KAT mismatches numpy twin vs reference plot = {mism}; "
              f"ambiguous raw pixels = {int(amb.sum())}; sum u={u.sum()!r} v={v.sum()!r}")
        assert mism == 0, "numpy twin does not reproduce the reference plot"
        np.savez_compressed(f"{HERE}/kat_{tag}.npz", labels=lab_ref, ambiguous=amb)
        meta["kat"][tag] = {"sum_u": float(u.sum()), "sum_v": float(v.sum()),
                            "window": 5, "iters": 100, "alpha": 1.0,
                            "n_green": int((lab_ref == 1).sum()),
                            "n_red": int((lab_ref == 2).sum()),
                            "n_ambiguous": int(amb.sum())}
        if tag == "000050":
            # a small BGR crop for the cvtColor test (input = BGR as imread gives)
            crop = prev_rgb[100:132, 400:448][..., ::-1]
            np.savez_compressed(f"{HERE}/bgr_crop.npz", bgr=crop,
                                gray=gray15(crop[..., ::-1]))

    g0, g1 = grays["000050"]
    # 64x48 crop (cols x rows): u,v for several windows / iteration counts
    c0, c1 = g0[150:198, 600:664], g1[150:198, 600:664]
    small = {"I0": c0, "I1": c1}
    gx, gy, gt = np_gradients(c0, c1)
    small.update(gx=gx, gy=gy, gt=gt)
    cases = [(5, 1), (5, 10), (5, 100), (3, 1), (3, 10), (3, 100),
             (4, 10), (1, 10), (2, 10), (7, 10), (9, 10)]
    for w, n in cases:
        u, v = np_flow(c0, c1, w, n, 1.0)
        small[f"u_w{w}_n{n}"], small[f"v_w{w}_n{n}"] = u, v
    # alpha != 1
    u, v = np_flow(c0, c1, 5, 10, 15.0)
    small["u_w5_n10_a15"], small["v_w5_n10_a15"] = u, v
    np.savez_compressed(f"{HERE}/crop64x48.npz", **small)

    # config 1: KITTI 000050 centre crop rows [59,315) x cols [493,749)
    c0, c1 = g0[59:315, 493:749], g1[59:315, 493:749]
    u, v = np_flow(c0, c1, 5, 100, 1.0)
    np.savez_compressed(f"{HERE}/crop256.npz", I0=c0, I1=c1, u=u, v=v)
    meta["crop256"] = {"rows": [59, 315], "cols": [493, 749], "window": 5,
                       "iters": 100, "alpha": 1.0}
    with open(f"{HERE}/golden.json", "w") as f:
        json.dump(meta, f, indent=2)
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
