"""GPU input path: main.cpp:13-14 BGR->gray on the device
feeding K1.  Integer work, so everything is checked bit-exactly: against the
reference-pinned fixture (tests/golden/bgr_crop.npz, gray made by the OpenCV
4.x formula that reproduces the reference plots), the host converter and the
oracle."""
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN


@pytest.fixture(scope="module")
def hs():
    import hsflow
    return hsflow


def _bgr(rows, cols, seed=3, batch=None):
    rng = np.random.default_rng(seed)
    shape = (rows, cols, 3) if batch is None else (batch, rows, cols, 3)
    return rng.integers(0, 256, shape, dtype=np.uint8)


def test_oracle_gray_matches_fixture():
    z = np.load(os.path.join(GOLDEN, "bgr_crop.npz"))
    assert np.array_equal(oracle.bgr_to_gray(z["bgr"]), z["gray"])


@pytest.mark.gpu
def test_device_gray_matches_fixture(hs):
    import torch
    z = np.load(os.path.join(GOLDEN, "bgr_crop.npz"))
    g = hs.bgr_to_gray_device(torch.from_numpy(z["bgr"]).cuda())
    assert np.array_equal(g.cpu().numpy(), z["gray"])


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(1, 1), (3, 5), (7, 37), (64, 128), (33, 1001),
                                   (70001, 9), (65536, 8)])
def test_device_gray_matches_host_and_oracle(hs, shape):
    import torch
    bgr = _bgr(*shape)
    g = hs.bgr_to_gray_device(torch.from_numpy(bgr).cuda()).cpu().numpy()
    assert np.array_equal(g, hs.bgr_to_gray(bgr))
    assert np.array_equal(g, oracle.bgr_to_gray(bgr))


@pytest.mark.gpu
def test_device_gray_batch(hs):
    import torch
    bgr = _bgr(19, 44, batch=3)
    g = hs.bgr_to_gray_device(torch.from_numpy(bgr).cuda()).cpu().numpy()
    for k in range(3):
        assert np.array_equal(g[k], oracle.bgr_to_gray(bgr[k]))


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(61, 83), (96, 128)])
def test_flow_bgr_equals_gray_flow(hs, shape):
    """hsflow_flow_bgr == getFlow(preprocess(frame)) bit for bit, and within
    tolerance of the oracle's main.cpp path."""
    b0 = _bgr(*shape, seed=11)
    b1 = np.roll(b0, (1, 2), (0, 1))
    ctx = hs.Context(0)
    u, v = ctx.flow_bgr(b0, b1, 5, 25, 1.0)
    g0, g1 = hs.bgr_to_gray(b0), hs.bgr_to_gray(b1)
    ug, vg = ctx.flow(g0, g1, 5, 25, 1.0)
    # ROI (non-dense BGR rows) honours the step
    big0 = np.zeros((shape[0], shape[1] + 7, 3), np.uint8)
    big1 = np.zeros_like(big0)
    big0[:, :shape[1]] = b0
    big1[:, :shape[1]] = b1
    ur, vr = ctx.flow_bgr(big0[:, :shape[1]], big1[:, :shape[1]], 5, 25, 1.0)
    ctx.close()
    assert np.array_equal(u, ug) and np.array_equal(v, vg)
    assert np.array_equal(ur, ug) and np.array_equal(vr, vg)
    uo, vo = oracle.flow(oracle.bgr_to_gray(b0), oracle.bgr_to_gray(b1), 5, 25, 1.0)
    from conftest import norm_rel_err
    assert norm_rel_err(u, uo) <= 1e-4 and norm_rel_err(v, vo) <= 1e-4


@pytest.mark.gpu
def test_flow_bgr_argument_errors(hs):
    ctx = hs.Context(0)
    with pytest.raises(hs.HsflowError):
        ctx.flow_bgr(_bgr(8, 8), _bgr(8, 9), 5, 1, 1.0)
    with pytest.raises(hs.HsflowError):
        ctx.flow_bgr(_bgr(8, 8)[..., 0], _bgr(8, 8)[..., 0], 5, 1, 1.0)
    ctx.close()
