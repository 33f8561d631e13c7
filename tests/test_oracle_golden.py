"""Pin the CPU oracle (oracle/hs_oracle.c) to the golden fixtures.

The fixtures come from tests/golden/make_golden.py: an independent numpy
restatement, itself checked pixel-exactly against the reference's own output
plots (HornSchunckOF/img/resimage/*hsbresenhamLineFlow.png).  Here the C
oracle is checked against (a) the same reference plots (KAT) and (b) the
numpy golden (u, v) arrays.
"""
import numpy as np
import pytest

import oracle
from conftest import kat_labels, norm_rel_err


def plot_labels(u, v):
    rows, cols = u.shape
    canvas = np.zeros((rows, cols, 3), np.uint8)
    img = oracle.plot_bresenham(canvas, u, v, 20, 20.0, 5)
    lab = np.zeros((rows, cols), np.uint8)
    lab[(img[..., 0] == 0) & (img[..., 1] == 255) & (img[..., 2] == 0)] = 1
    lab[(img[..., 0] == 0) & (img[..., 1] == 0) & (img[..., 2] == 255)] = 2
    return lab


def test_bgr_to_gray_matches_fixture():
    from conftest import GOLDEN
    import os
    z = np.load(os.path.join(GOLDEN, "bgr_crop.npz"))
    assert np.array_equal(oracle.bgr_to_gray(z["bgr"]), z["gray"])


def test_gradients_exact(crop_small):
    gx, gy, gt = oracle.gradients(crop_small["I0"], crop_small["I1"])
    assert np.array_equal(gx, crop_small["gx"])
    assert np.array_equal(gy, crop_small["gy"])
    assert np.array_equal(gt, crop_small["gt"])
    assert np.abs(gx).max() <= 1020 and np.abs(gt).max() <= 255


@pytest.mark.parametrize("w,n", [(5, 1), (5, 10), (5, 100), (3, 1), (3, 10), (3, 100),
                                 (4, 10), (1, 10), (2, 10), (7, 10), (9, 10)])
def test_flow_matches_numpy_golden(crop_small, w, n):
    u, v = oracle.flow(crop_small["I0"], crop_small["I1"], w, n, 1.0)
    assert norm_rel_err(u, crop_small[f"u_w{w}_n{n}"]) < 1e-12
    assert norm_rel_err(v, crop_small[f"v_w{w}_n{n}"]) < 1e-12


def test_flow_alpha(crop_small):
    u, v = oracle.flow(crop_small["I0"], crop_small["I1"], 5, 10, 15.0)
    assert norm_rel_err(u, crop_small["u_w5_n10_a15"]) < 1e-12
    assert norm_rel_err(v, crop_small["v_w5_n10_a15"]) < 1e-12


def test_config1_crop256(crop256):
    u, v = oracle.flow(crop256["I0"], crop256["I1"], 5, 100, 1.0, nthreads=4)
    assert norm_rel_err(u, crop256["u"]) < 1e-12
    assert norm_rel_err(v, crop256["v"]) < 1e-12


def test_jacobi_continuation(crop_small):
    """10 iterations == 4 then 6 from the intermediate state."""
    gx, gy, gt = oracle.gradients(crop_small["I0"], crop_small["I1"])
    z = np.zeros_like(gx)
    u4, v4 = oracle.jacobi(gx, gy, gt, z, z, 5, 4, 1.0)
    u, v = oracle.jacobi(gx, gy, gt, u4, v4, 5, 6, 1.0)
    assert np.array_equal(u, crop_small["u_w5_n10"]) or \
        norm_rel_err(u, crop_small["u_w5_n10"]) < 1e-12


@pytest.mark.parametrize("tag", ["000050", "000040"])
def test_reference_plot_kat(kitti, golden_meta, tag):
    """The reference's own output (arrow plot after ws=5, 100 it, alpha=1,
    main.cpp:94-104) is reproduced pixel-exactly from the oracle's (u, v)."""
    I0, I1 = kitti[tag]
    u, v = oracle.flow(I0, I1, 5, 100, 1.0, nthreads=8)
    meta = golden_meta["kat"][tag]
    assert abs(u.sum() - meta["sum_u"]) < 1e-6 * abs(meta["sum_u"])
    assert abs(v.sum() - meta["sum_v"]) < 1e-6 * abs(meta["sum_v"])
    ref, amb = kat_labels(tag)
    lab = plot_labels(u, v)
    assert int(np.count_nonzero((lab != ref) & ~amb)) == 0


def test_reflect101_tiny_images():
    """Sobel on 1- and 2-pixel-wide images (borderInterpolate len==1 -> 0)."""
    for shape in [(1, 1), (1, 5), (5, 1), (2, 2), (2, 7)]:
        I0 = np.arange(np.prod(shape), dtype=np.float64).reshape(shape) * 7 % 255
        I1 = I0[::-1, ::-1].copy()
        from golden.make_golden import np_gradients
        gx, gy, gt = oracle.gradients(I0, I1)
        ex, ey, et = np_gradients(I0, I1)
        assert np.array_equal(gx, ex) and np.array_equal(gy, ey) and np.array_equal(gt, et)
