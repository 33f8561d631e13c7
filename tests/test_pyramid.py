"""Config 5 (north_star): coarse-to-fine pyramid warm start + fp16 inputs.

HornSchunckOF has no pyramid, so there is no reference output to pin this
against: the C oracle's pyramid (oracle/hs_oracle.c hso_pyrdown /
hso_flow_pyramid) is checked here against an independent numpy restatement
of the same design precedent (BMOpticalFlow/.../OpticalFlow/
MultiResolution.cpp:9-97 Pyramider, OpticalFlow.cpp:197-210
Add_VectorOffset) built on the already-pinned per-level oracle pieces
(gradients, jacobi).  "Parity unpinned" w.r.t. the reference for levels > 1;
levels = 1 is the pinned getFlow path.  The GPU path is then checked against
the oracle with the module's usual tolerance (max|d|/max|ref| <= 1e-4) and
bit-exactly for integer work (level images of integer-valued pairs).
"""
import numpy as np
import pytest

import oracle
from conftest import norm_rel_err

TOL = 1e-4
W5 = np.array([2.0, 5.0, 4.0, 5.0, 2.0])  # (a/2, 1/2, a, 1/2, a/2) * 18, a = 0.4


def _refl101(p, n):
    if n == 1:
        return np.zeros_like(p)
    p = np.abs(p)
    p = np.where(p >= n, 2 * (n - 1) - p, p)
    return np.abs(p)


def pyrdown_np(img, rnd):
    """Independent twin of hso_pyrdown: separable 5-tap, stride 2, reflect-101."""
    a = np.asarray(img, np.float64)
    r, c = a.shape
    r2, c2 = (r + 1) // 2, (c + 1) // 2
    ys = _refl101(2 * np.arange(r2)[:, None] + np.arange(5)[None, :] - 2, r)  # r2 x 5
    xs = _refl101(2 * np.arange(c2)[:, None] + np.arange(5)[None, :] - 2, c)  # c2 x 5
    h = np.einsum("rxn,n->rx", a[:, xs], W5)          # r x c2
    S = np.einsum("ymx,m->yx", h[ys, :], W5)          # r2 x c2
    return np.floor((S + 162.0) / 324.0) if rnd else S / 324.0


def pyramid_np(I0, I1, levels, w, n, alpha):
    a, b = np.asarray(I0, np.float64), np.asarray(I1, np.float64)
    rnd = bool(np.all(a == np.floor(a)) and np.all(b == np.floor(b)) and a.min() >= 0
               and b.min() >= 0 and a.max() <= 255 and b.max() <= 255)
    P = [(a, b)]
    for _ in range(1, levels):
        P.append((pyrdown_np(P[-1][0], rnd), pyrdown_np(P[-1][1], rnd)))
    u = v = None
    for lv in range(levels - 1, -1, -1):
        p0, p1 = P[lv]
        if u is None:
            u0 = np.zeros_like(p0)
            v0 = np.zeros_like(p0)
        else:  # OpticalFlow.cpp:205-206, nearest projection x 2
            u0 = 2.0 * np.repeat(np.repeat(u, 2, 0), 2, 1)[:p0.shape[0], :p0.shape[1]]
            v0 = 2.0 * np.repeat(np.repeat(v, 2, 0), 2, 1)[:p0.shape[0], :p0.shape[1]]
        gx, gy, gt = oracle.gradients(p0, p1)
        u, v = oracle.jacobi(gx, gy, gt, u0, v0, w, n, alpha)
    return u, v


def _pair(rows, cols, seed=7, integral=True):
    rng = np.random.default_rng(seed)
    I0 = rng.integers(0, 256, (rows, cols)).astype(np.float64)
    # smooth-ish second frame: shift + noise
    I1 = np.clip(np.roll(I0, (1, -2), (0, 1)) + rng.integers(-3, 4, (rows, cols)), 0, 255)
    if not integral:
        I0 = I0 + 0.25
    return I0, I1


# ------------------------------------------------------------------ CPU tests
@pytest.mark.parametrize("shape", [(1, 1), (1, 6), (2, 3), (5, 7), (17, 33), (48, 64)])
@pytest.mark.parametrize("rnd", [True, False])
def test_oracle_pyrdown_matches_numpy_twin(shape, rnd):
    I0, _ = _pair(*shape, integral=rnd)
    got = oracle.pyrdown(I0, rnd)
    ref = pyrdown_np(I0, rnd)
    assert got.shape == ((shape[0] + 1) // 2, (shape[1] + 1) // 2)
    if rnd:
        assert np.array_equal(got, ref)
        assert got.min() >= 0 and got.max() <= 255
    else:
        assert np.allclose(got, ref, rtol=0, atol=1e-12)


def test_oracle_pyrdown_preserves_constants():
    # the normalised kernel has unit DC gain (MultiResolution.cpp:58-63)
    img = np.full((9, 14), 137.0)
    assert np.array_equal(oracle.pyrdown(img, True), np.full((5, 7), 137.0))


def test_oracle_integer_pair_rule():
    I0, I1 = _pair(6, 9)
    assert oracle.integer_pair(I0, I1)
    assert not oracle.integer_pair(I0 + 0.5, I1)
    J = I1.copy()
    J[0, 0] = 256
    assert not oracle.integer_pair(I0, J)


def test_oracle_pyramid_one_level_is_getflow(crop_small):
    I0, I1 = crop_small["I0"], crop_small["I1"]
    u1, v1 = oracle.flow_pyramid(I0, I1, 1, 5, 10, 1.0)
    u, v = oracle.flow(I0, I1, 5, 10, 1.0)
    assert np.array_equal(u1, u) and np.array_equal(v1, v)


@pytest.mark.parametrize("shape,levels", [((48, 64), 3), ((37, 53), 3), ((20, 9), 4)])
@pytest.mark.parametrize("integral", [True, False])
def test_oracle_pyramid_matches_numpy_twin(shape, levels, integral):
    I0, I1 = _pair(*shape, integral=integral)
    u, v = oracle.flow_pyramid(I0, I1, levels, 5, 7, 1.0)
    ur, vr = pyramid_np(I0, I1, levels, 5, 7, 1.0)
    assert norm_rel_err(u, ur) <= 1e-12 and norm_rel_err(v, vr) <= 1e-12


# ------------------------------------------------------------------ GPU tests
@pytest.fixture(scope="module")
def hs():
    import hsflow
    return hsflow


def _dev_pyr(hs, I0, I1, levels, w, n, alpha=1.0, torch_dtype=None):
    import torch
    t0 = torch.from_numpy(np.ascontiguousarray(I0)).cuda()
    t1 = torch.from_numpy(np.ascontiguousarray(I1)).cuda()
    if torch_dtype is not None:
        t0, t1 = t0.to(torch_dtype), t1.to(torch_dtype)
    u, v = hs.flow_pyramid_device(t0, t1, levels, w, n, alpha)
    torch.cuda.synchronize()
    return u.cpu().numpy(), v.cpu().numpy()


@pytest.mark.gpu
def test_f16_inputs_match_f32_bitwise(hs):
    """Config 5 stores the frames as fp16: integer-valued fp16 frames give
    exactly the f32 result (same packed gradients)."""
    import torch
    I0, I1 = hs.synth_pair(1003, 200, 331)
    t0, t1 = torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()
    a = hs.flow_device(t0, t1, 5, 40, 1.0)
    b = hs.flow_device(t0.half(), t1.half(), 5, 40, 1.0)
    torch.cuda.synchronize()
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    uo, vo = oracle.flow(I0, I1, 5, 40, 1.0, nthreads=8)
    assert norm_rel_err(b[0].cpu().numpy(), uo) <= TOL
    assert norm_rel_err(b[1].cpu().numpy(), vo) <= TOL


@pytest.mark.gpu
def test_f16_host_api(hs):
    I0, I1 = hs.synth_pair(1004, 64, 96)
    ctx = hs.Context(0)
    u16, v16 = ctx.flow(I0.astype(np.float16), I1.astype(np.float16), 5, 20, 1.0)
    u32, v32 = ctx.flow(I0, I1, 5, 20, 1.0)
    ctx.close()
    assert np.array_equal(u16, u32) and np.array_equal(v16, v32)


@pytest.mark.gpu
def test_pyramid_one_level_is_flow_device_bitwise(hs):
    import torch
    I0, I1 = hs.synth_pair(1005, 130, 250)
    t0, t1 = torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()
    a = hs.flow_device(t0, t1, 5, 30, 1.0)
    b = hs.flow_pyramid_device(t0, t1, 1, 5, 30, 1.0)
    torch.cuda.synchronize()
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(96, 160), (97, 161), (45, 300), (5, 3)])
@pytest.mark.parametrize("levels", [2, 3])
@pytest.mark.parametrize("w", [3, 5])
def test_pyramid_against_oracle(hs, shape, levels, w):
    I0, I1 = hs.synth_pair(1006, *shape)
    u, v = _dev_pyr(hs, I0, I1, levels, w, 25)
    uo, vo = oracle.flow_pyramid(I0, I1, levels, w, 25, 1.0, nthreads=8)
    assert norm_rel_err(u, uo) <= TOL and norm_rel_err(v, vo) <= TOL


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["u8", "f16", "f32_nonint"])
def test_pyramid_input_kinds(hs, kind):
    import torch
    I0, I1 = hs.synth_pair(1007, 150, 222)
    if kind == "u8":
        a, b, td = I0.astype(np.uint8), I1.astype(np.uint8), None
    elif kind == "f16":
        a, b, td = I0, I1, torch.float16
    else:
        a, b, td = I0 * np.float32(0.9) + np.float32(0.3), I1, None
    u, v = _dev_pyr(hs, a, b, 3, 5, 30, torch_dtype=td)
    uo, vo = oracle.flow_pyramid(np.asarray(a, np.float64), np.asarray(b, np.float64), 3, 5,
                                 30, 1.0, nthreads=8)
    assert norm_rel_err(u, uo) <= TOL and norm_rel_err(v, vo) <= TOL


@pytest.mark.gpu
def test_pyramid_host_equals_device(hs):
    I0, I1 = hs.synth_pair(1008, 120, 200)
    ctx = hs.Context(0)
    uh, vh = ctx.flow_pyramid(I0, I1, 3, 5, 20, 1.0, out_dtype=np.float32)
    ctx.close()
    ud, vd = _dev_pyr(hs, I0, I1, 3, 5, 20)
    assert np.array_equal(uh, ud) and np.array_equal(vh, vd)


@pytest.mark.gpu
def test_pyramid_batch_equals_single(hs):
    import torch
    pairs = [hs.synth_pair(1010 + k, 77, 140) for k in range(3)]
    t0 = torch.stack([torch.from_numpy(p[0]) for p in pairs]).cuda()
    t1 = torch.stack([torch.from_numpy(p[1]) for p in pairs]).cuda()
    ub, vb = hs.flow_pyramid_device(t0, t1, 3, 5, 15, 1.0)
    for k in range(3):
        us, vs = hs.flow_pyramid_device(t0[k].contiguous(), t1[k].contiguous(), 3, 5, 15, 1.0)
        assert torch.equal(ub[k], us) and torch.equal(vb[k], vs)


@pytest.mark.gpu
def test_pyramid_argument_errors(hs):
    import torch
    t = torch.zeros(8, 8, device="cuda")
    for levels in (0, hs.MAX_LEVELS + 1):
        with pytest.raises(hs.HsflowError):
            hs.flow_pyramid_device(t, t, levels, 5, 1, 1.0)
    assert hs.pyramid_level_size(4320, 7680, 2) == (1080, 1920)
    assert hs.pyramid_level_size(5, 3, 2) == (2, 1)


@pytest.mark.gpu
def test_config5_8k_fp16_pyramid(hs):
    """Config 5 shape: 7680x4320 fp16 pair, 3 levels.  Short per-level runs
    against the oracle at full size, fp16 == f32 bitwise, finite output."""
    import torch
    I0, I1 = hs.synth_pair(1000, 4320, 7680)
    t0, t1 = torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()
    u16, v16 = hs.flow_pyramid_device(t0.half(), t1.half(), 3, 5, 12, 1.0)
    u32, v32 = hs.flow_pyramid_device(t0, t1, 3, 5, 12, 1.0)
    torch.cuda.synchronize()
    assert torch.equal(u16, u32) and torch.equal(v16, v32)
    assert bool(torch.isfinite(u16).all()) and bool(torch.isfinite(v16).all())
    uo, vo = oracle.flow_pyramid(I0, I1, 3, 5, 12, 1.0, nthreads=16)
    assert norm_rel_err(u16.cpu().numpy(), uo) <= TOL
    assert norm_rel_err(v16.cpu().numpy(), vo) <= TOL
