"""GPU parity tests: the HIP path (libhsflow.so, through its C ABI) against the
CPU float64 oracle (oracle/hs_oracle.c) and the golden fixtures.

Tolerance (north_star: "within 1e-4 relative fp32"; SURVEY §8c form):
    max|got - ref| / max|ref| <= 1e-4        (TOL below)
Integer work (gradients, packing, plot KAT label maps, K-invariance, batch
vs single) is checked bit-exactly.
"""
import numpy as np
import pytest

import oracle
from conftest import kat_labels, norm_rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-4


@pytest.fixture(scope="module")
def hs():
    import hsflow
    return hsflow


@pytest.fixture(scope="module")
def ctx(hs):
    c = hs.Context(0)
    yield c
    c.close()


def _oracle_flow(I0, I1, w, n, alpha=1.0):
    return oracle.flow(I0, I1, w, n, alpha, nthreads=8)


def test_native_library_is_loaded(hs, ctx):
    with open("/proc/self/maps") as f:
        maps = f.read()
    assert "libhsflow.so" in maps


@pytest.mark.parametrize("w,n", [(5, 1), (5, 10), (5, 100), (3, 1), (3, 10), (3, 100),
                                 (4, 10), (1, 10), (2, 10), (7, 10), (9, 10)])
def test_crop_matches_golden(hs, ctx, crop_small, w, n):
    u, v = ctx.flow(crop_small["I0"], crop_small["I1"], w, n, 1.0)
    assert u.dtype == np.float64  # CV_64FC1 like the reference
    assert norm_rel_err(u, crop_small[f"u_w{w}_n{n}"]) <= TOL
    assert norm_rel_err(v, crop_small[f"v_w{w}_n{n}"]) <= TOL


def test_alpha(hs, ctx, crop_small):
    u, v = ctx.flow(crop_small["I0"], crop_small["I1"], 5, 10, 15.0)
    assert norm_rel_err(u, crop_small["u_w5_n10_a15"]) <= TOL
    assert norm_rel_err(v, crop_small["v_w5_n10_a15"]) <= TOL


def test_config1_crop256(hs, crop256):
    """BASELINE config 1: KITTI 000050 centre crop, ws 5, alpha 1, 100 it."""
    u, v = hs.hornSchunck(5, 100, 1.0).getFlow(crop256["I0"], crop256["I1"])
    assert norm_rel_err(u, crop256["u"]) <= TOL
    assert norm_rel_err(v, crop256["v"]) <= TOL


@pytest.mark.parametrize("tag", ["000050", "000040"])
def test_reference_plot_kat(hs, kitti, golden_meta, tag):
    """The reference's own arrow plot (main.cpp:94-104 -> plotFlow.cpp:68-88)
    is reproduced pixel-exactly from the GPU (u, v)."""
    I0, I1 = kitti[tag]
    hsobj = hs.hornSchunck(5, 100, 1.0)
    u, v = hsobj.getFlow(I0, I1)
    uo, vo = _oracle_flow(I0, I1, 5, 100)
    assert norm_rel_err(u, uo) <= TOL and norm_rel_err(v, vo) <= TOL
    meta = golden_meta["kat"][tag]
    assert abs(u.sum() - meta["sum_u"]) <= 1e-4 * abs(meta["sum_u"])
    assert abs(v.sum() - meta["sum_v"]) <= 1e-4 * abs(meta["sum_v"])
    canvas = np.zeros(I0.shape + (3,), np.uint8)
    img = oracle.plot_bresenham(canvas, u, v, 20, 20.0, 5)
    lab = np.zeros(I0.shape, np.uint8)
    lab[(img[..., 0] == 0) & (img[..., 1] == 255) & (img[..., 2] == 0)] = 1
    lab[(img[..., 0] == 0) & (img[..., 1] == 0) & (img[..., 2] == 255)] = 2
    ref, amb = kat_labels(tag)
    assert int(np.count_nonzero((lab != ref) & ~amb)) == 0


@pytest.mark.parametrize("dtype", [np.uint8, np.float32, np.float64])
def test_gradients_exact(hs, ctx, kitti, dtype):
    I0, I1 = kitti["000050"]
    gx, gy, gt = ctx.gradients(I0.astype(dtype), I1.astype(dtype))
    ex, ey, et = oracle.gradients(I0, I1)
    assert np.array_equal(gx, ex) and np.array_equal(gy, ey) and np.array_equal(gt, et)


def test_get_gradients_mirror(hs, crop_small):
    gx, gy, gt = hs.hornSchunck(5, 1, 1.0).getGradients(crop_small["I0"], crop_small["I1"])
    assert np.array_equal(gx, crop_small["gx"]) and np.array_equal(gt, crop_small["gt"])


@pytest.mark.parametrize("shape", [(1, 1), (1, 7), (7, 1), (2, 2), (3, 130), (130, 3),
                                   (47, 63), (65, 65), (49, 300), (300, 49), (97, 129)])
@pytest.mark.parametrize("w", [3, 5])
def test_ragged_and_tiny_shapes(hs, ctx, shape, w):
    I0, I1 = hs.synth_pair(1234, *shape, dtype=np.uint8)
    u, v = ctx.flow(I0, I1, w, 13, 1.0)
    uo, vo = _oracle_flow(I0, I1, w, 13)
    if np.abs(uo).max() == 0:
        assert np.abs(u).max() == 0
    else:
        assert norm_rel_err(u, uo) <= TOL and norm_rel_err(v, vo) <= TOL


@pytest.mark.parametrize("w", [1, 2, 4, 6, 8, 10, 11, 15, 21])
def test_all_window_sizes(hs, ctx, w):
    I0, I1 = hs.synth_pair(77, 45, 70, dtype=np.uint8)
    u, v = ctx.flow(I0, I1, w, 7, 1.0)
    uo, vo = _oracle_flow(I0, I1, w, 7)
    assert norm_rel_err(u, uo) <= TOL and norm_rel_err(v, vo) <= TOL


@pytest.mark.parametrize("kernel", [0, 2, 4])  # automatic, K2 tiles, K4 strips (w 3, 5)
@pytest.mark.parametrize("w", [3, 5, 6, 9])
def test_alpha_zero_nan_pattern_matches_the_oracle(hs, w, kernel):
    """alpha = 0 is a legal hornSchunck argument.  The reference then divides
    by Ix^2 + Iy^2 (hornSchunck.cpp:63-68), which is 0 at every image corner
    (reflect-101 Sobel: Ix = 0 on the first and last column, Iy on the first
    and last row), so NaN appears there and spreads through the window sums.
    The GPU must give NaN exactly where the oracle does and match it
    elsewhere: the strip/tile columns outside the image must stay 0, not
    0 * rsq(0) = NaN (hsflow_device.h alpha2_cols)."""
    import torch
    I0, I1 = hs.synth_pair(321, 70, 300)  # several K4 strips / K2 tiles across
    uo, vo = _oracle_flow(I0, I1, w, 6, alpha=0.0)
    assert not np.isfinite(uo).all() and np.isfinite(uo).mean() > 0.5
    hs.set_jacobi_kernel(kernel)
    try:
        # a batch of two (the K4 batch rules) and the single pair
        t0 = torch.from_numpy(np.stack([I0, I0])).cuda()
        t1 = torch.from_numpy(np.stack([I1, I1])).cuda()
        ub, vb = hs.flow_device(t0, t1, w, 6, 0.0)
        torch.cuda.synchronize()
        us, vs = hs.flow_device(t0[:1], t1[:1], w, 6, 0.0)
        torch.cuda.synchronize()
    finally:
        hs.set_jacobi_kernel(0)
    for got_u, got_v in ((ub[0], vb[0]), (ub[1], vb[1]), (us[0], vs[0])):
        for got, ref in ((got_u.cpu().numpy(), uo), (got_v.cpu().numpy(), vo)):
            fin = np.isfinite(ref)
            assert np.array_equal(np.isfinite(got), fin)
            d = np.abs(got[fin].astype(np.float64) - ref[fin])
            assert d.max() / np.abs(ref[fin]).max() <= TOL


def test_zero_iterations_gives_zero_flow(hs, ctx, crop_small):
    u, v = ctx.flow(crop_small["I0"], crop_small["I1"], 5, 0, 1.0)
    assert not u.any() and not v.any()


def test_non_integral_f32_inputs_use_f32_gradients(hs, ctx):
    I0, I1 = hs.synth_pair(5, 150, 170)
    rng = np.random.default_rng(0)
    I0 = (I0 + rng.uniform(-0.5, 0.5, I0.shape)).astype(np.float32)
    I1 = (I1 * 0.731).astype(np.float32)
    for w, n in [(5, 40), (3, 40), (7, 9)]:
        u, v = ctx.flow(I0, I1, w, n, 1.0)
        uo, vo = _oracle_flow(I0.astype(np.float64), I1.astype(np.float64), w, n)
        assert norm_rel_err(u, uo) <= TOL and norm_rel_err(v, vo) <= TOL


def test_roi_input_honours_row_step(hs, ctx, kitti):
    """cv::Mat ROIs are non-continuous (hornSchunck.cpp takes Mat by value)."""
    I0, I1 = kitti["000040"]
    roi0, roi1 = I0[30:130, 100:333], I1[30:130, 100:333]
    assert not roi0.flags["C_CONTIGUOUS"]
    u, v = ctx.flow(roi0, roi1, 5, 20, 1.0)
    u2, v2 = ctx.flow(np.ascontiguousarray(roi0), np.ascontiguousarray(roi1), 5, 20, 1.0)
    assert np.array_equal(u, u2) and np.array_equal(v, v2)


def test_size_mismatch_raises(hs, ctx):
    with pytest.raises(hs.HsflowError) as e:
        ctx.flow(np.zeros((4, 4), np.uint8), np.zeros((4, 5), np.uint8), 5, 1, 1.0)
    assert e.value.status == hs.HSFLOW_ERR_SIZE


def test_f32_output(hs, ctx, crop_small):
    u32, _ = ctx.flow(crop_small["I0"], crop_small["I1"], 5, 10, 1.0, out_dtype=np.float32)
    u64, _ = ctx.flow(crop_small["I0"], crop_small["I1"], 5, 10, 1.0)
    assert u32.dtype == np.float32 and np.array_equal(u32.astype(np.float64), u64)


# --------------------------------------------------------------- invariances
def _device_flow(hs, I0, I1, w, n, kb):
    import torch
    hs.set_iters_per_launch(kb)
    try:
        u, v = hs.flow_device(I0, I1, w, n, 1.0)
        torch.cuda.synchronize()
    finally:
        hs.set_iters_per_launch(0)
    return u.cpu().numpy(), v.cpu().numpy()


KBS = (2, 3, 4, 5, 6, 8)


@pytest.mark.parametrize("dtype", ["uint8", "float32"])
@pytest.mark.parametrize("cols", [517, 518])  # odd: dword path, even: 8-byte pairs
def test_blocking_depth_is_bit_invariant(hs, dtype, cols):
    """Temporal blocking (KB iterations per launch) changes no bit."""
    import torch
    I0, I1 = hs.synth_pair(1001, 300, cols, dtype=np.uint8)
    t0 = torch.from_numpy(I0.astype(dtype)).cuda()
    t1 = torch.from_numpy(I1.astype(dtype)).cuda()
    ref = _device_flow(hs, t0, t1, 5, 23, 1)
    for kb in KBS:
        got = _device_flow(hs, t0, t1, 5, 23, kb)
        assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]), kb
    ref3 = _device_flow(hs, t0, t1, 3, 19, 1)
    for kb in KBS:
        got = _device_flow(hs, t0, t1, 3, 19, kb)
        assert np.array_equal(got[0], ref3[0]), kb


@pytest.mark.parametrize("w", [4, 6, 7, 8, 9])
@pytest.mark.parametrize("cols", [301, 302])
@pytest.mark.parametrize("integral", [True, False])
def test_blocking_depth_bit_invariant_wide_windows(hs, w, cols, integral):
    """Windows 3..9 share the workgroup kernel (generic horizontal/vertical
    trees): every supported blocking depth gives the same bits, and the
    result matches the float64 oracle."""
    import torch
    I0, I1 = hs.synth_pair(77, 190, cols)
    if not integral:
        I0 = I0 * np.float32(0.9) + np.float32(0.35)
    t0, t1 = torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()
    n = 13
    ref = _device_flow(hs, t0, t1, w, n, 1)
    for kb in (2, 3, 4, 5, 6, 8):
        if kb * (w - 1) > 32:
            continue
        got = _device_flow(hs, t0, t1, w, n, kb)
        assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]), kb
    uo, vo = oracle.flow(I0, I1, w, n, 1.0, nthreads=8)
    assert norm_rel_err(ref[0], uo) <= TOL and norm_rel_err(ref[1], vo) <= TOL


@pytest.mark.parametrize("cols", [333, 334])
def test_blocking_depth_bit_invariant_f32_gradients(hs, cols):
    import torch
    I0, I1 = hs.synth_pair(9, 200, cols)
    I0 = I0 + np.float32(0.25)
    t0, t1 = torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()
    ref = _device_flow(hs, t0, t1, 5, 11, 1)
    for kb in KBS:
        got = _device_flow(hs, t0, t1, 5, 11, kb)
        assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]), kb
    uo, vo = oracle.flow(I0, I1, 5, 11, 1.0, nthreads=8)
    assert norm_rel_err(ref[0], uo) <= TOL and norm_rel_err(ref[1], vo) <= TOL


def test_f32_gradient_path_equals_packed_for_integer_frames(hs):
    """The f32-gradient loader and the packed loader feed the same operator:
    integer-valued frames give the same bits through either."""
    import torch
    I0, I1 = hs.synth_pair(21, 150, 260)
    t0, t1 = torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()
    a = hs.flow_device(t0, t1, 5, 17, 1.0)
    ws = hs.alloc_workspace(150, 260, 1)
    hs.gradients_device(t0, t1, ws)
    # force the f32 planes: set the pair's flag word (last 4 B of the workspace
    # layout is not guaranteed, so mark it through a non-integral twin instead)
    J0 = t0.clone()
    J0[0, 0] += 0.5  # flags the pair; pixel (0,0) only affects its neighbourhood
    b = hs.flow_device(J0, t1, 5, 17, 1.0)
    torch.cuda.synchronize()
    ua, ub = a[0].cpu().numpy(), b[0].cpu().numpy()
    far = np.s_[40:, 60:]  # beyond 17 iterations x 2 px of influence
    assert np.array_equal(ua[far], ub[far])


def test_batch_equals_single_pairs(hs, ctx):
    import torch
    pairs = [hs.synth_pair(1000 + i, 130, 250) for i in range(3)]
    b0 = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    b1 = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    # pair 1 made non-integral: the batch mixes both gradient formats
    b0[1] += 0.5
    u, v = hs.flow_device(b0, b1, 5, 30, 1.0)
    torch.cuda.synchronize()
    for i in range(3):
        us, vs = hs.flow_device(b0[i].contiguous(), b1[i].contiguous(), 5, 30, 1.0)
        torch.cuda.synchronize()
        assert torch.equal(u[i], us) and torch.equal(v[i], vs)
        uo, vo = _oracle_flow(b0[i].cpu().numpy(), b1[i].cpu().numpy(), 5, 30)
        assert norm_rel_err(u[i].cpu().numpy(), uo) <= TOL


@pytest.mark.parametrize("w", [3, 5])
def test_single_pair_geometry_equals_batch(hs, w):
    """A single 1080p pair runs K2 at depth 8 in 16-wave x 8-row tiles (the
    fill-limited geometry); the same pair inside a batch of two runs other
    tiles and depths (K4 / 8-wave K2): the same bits."""
    import torch
    pairs = [hs.synth_pair(1000 + i, 1080, 1920) for i in range(2)]
    b0 = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    b1 = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    assert hs.iters_per_launch(1080, 1920, 1, w) == 8
    u, v = hs.flow_device(b0, b1, w, 40, 1.0)
    us, vs = hs.flow_device(b0[0].contiguous(), b1[0].contiguous(), w, 40, 1.0)
    torch.cuda.synchronize()
    assert torch.equal(u[0], us) and torch.equal(v[0], vs)


def test_warm_start_continuation_is_exact(hs):
    import torch
    I0, I1 = hs.synth_pair(3, 240, 320)
    t0, t1 = torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()
    u10, v10 = hs.flow_device(t0, t1, 5, 10, 1.0)
    ws = hs.alloc_workspace(240, 320)
    hs.gradients_device(t0, t1, ws)
    u = torch.empty_like(t0)
    v = torch.empty_like(t0)
    hs.jacobi_device(240, 320, 1, 5, 4, 1.0, u, v, ws)
    hs.jacobi_device(240, 320, 1, 5, 6, 1.0, u, v, ws, warm_start=True)
    torch.cuda.synchronize()
    assert torch.equal(u, u10) and torch.equal(v, v10)


# ------------------------------------------------------- full-size (configs)
def test_1080p_against_oracle(hs):
    """Config 2 shape (1920x1080 f32 synthetic), 30 iterations vs the oracle."""
    import torch
    I0, I1 = hs.synth_pair(1000, 1080, 1920)
    u, v = hs.flow_device(torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda(),
                          5, 30, 1.0)
    uo, vo = _oracle_flow(I0, I1, 5, 30)
    assert norm_rel_err(u.cpu().numpy(), uo) <= TOL
    assert norm_rel_err(v.cpu().numpy(), vo) <= TOL
    # Sobel scaling: the mean flow is ~dx/8 = 0.1875 (SURVEY §8d sanity)
    assert 0.05 < float(u.mean()) < 0.3


def test_config2_full_length_against_oracle(hs):
    """BASELINE configs[1] exactly: 1920x1080 f32 synthetic pair, alpha 1,
    300 iterations, w 5 -- GPU vs the float64 oracle at full length
    (oracle on 16 threads, ~15 s)."""
    import torch
    I0, I1 = hs.synth_pair(1000, 1080, 1920)
    u, v = hs.flow_device(torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda(),
                          5, 300, 1.0)
    uo, vo = oracle.flow(I0, I1, 5, 300, 1.0, nthreads=16)
    assert norm_rel_err(u.cpu().numpy(), uo) <= TOL
    assert norm_rel_err(v.cpu().numpy(), vo) <= TOL


def test_config3_full_length_against_oracle(hs):
    """BASELINE configs[2] exactly: 3840x2160 f32 synthetic pair, 500
    iterations, w 5 -- GPU vs the float64 oracle at full size and length
    (oracle on 16 threads, ~70 s)."""
    import torch
    I0, I1 = hs.synth_pair(1000, 2160, 3840)
    u, v = hs.flow_device(torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda(),
                          5, 500, 1.0)
    uo, vo = oracle.flow(I0, I1, 5, 500, 1.0, nthreads=16)
    eu, ev = norm_rel_err(u.cpu().numpy(), uo), norm_rel_err(v.cpu().numpy(), vo)
    print(f"config 3 full length: max|du|/max|u| = {eu:.2e}, dv {ev:.2e}")
    assert eu <= TOL and ev <= TOL


def test_4k_500_properties(hs):
    """Config 3 shape at full iteration count: size-independent properties
    (KB invariance, batch==single, finite, expected mean motion)."""
    import torch
    I0, I1 = hs.synth_pair(1000, 2160, 3840)
    t0, t1 = torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()
    a = _device_flow(hs, t0, t1, 5, 500, 4)
    b = _device_flow(hs, t0, t1, 5, 500, 2)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert np.isfinite(a[0]).all() and np.isfinite(a[1]).all()
    assert 0.05 < float(a[0].mean()) < 0.3
    # oracle check on a corner of the same frame (short run)
    s0, s1 = I0[:512, :768].copy(), I1[:512, :768].copy()
    us, _ = _device_flow(hs, torch.from_numpy(s0).cuda(), torch.from_numpy(s1).cuda(), 5, 40, 4)
    uo, _ = _oracle_flow(s0, s1, 5, 40)
    assert norm_rel_err(us, uo) <= TOL


# ------------------------------------------- C++ driver (main.cpp equivalent)
def _read_ppm(path):
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(maxsplit=4)
    w, h = int(parts[1]), int(parts[2])
    return np.frombuffer(parts[4], np.uint8, count=w * h * 3).reshape(h, w, 3)


def _read_fs_matrix(path):
    """Parse the cv::FileStorage YAML written by examples/hs_main.cpp."""
    txt = open(path).read()
    rows = int(txt.split("rows:")[1].split()[0])
    cols = int(txt.split("cols:")[1].split()[0])
    body = txt.split("data: [")[1].split("]")[0]
    vals = np.array([float(x) for x in body.replace("\n", " ").split(",")])
    return vals.reshape(rows, cols)


@pytest.mark.parametrize("tag", ["000050"])
def test_cpp_main_driver_reproduces_reference_plot(tmp_path, tag):
    """examples/hs_main (C++, include/hsflow.hpp over the C ABI) runs the
    reference main.cpp flow: reads the pair, getFlow(ws 5, 100 it, alpha 1),
    writes uMatrixHS.txt/vMatrixHS.txt and the arrow plot.  The plot's
    green/red pixels equal the reference's own plot (KAT)."""
    import os
    import subprocess
    from conftest import GOLDEN, ROOT
    exe = os.path.join(ROOT, "examples", "hs_main")
    assert os.path.exists(exe), "build with make -C cpp-optical-flow_amd"
    out = str(tmp_path / "r_")
    subprocess.check_call([exe, os.path.join(GOLDEN, f"kitti_{tag}_10.pgm"),
                           os.path.join(GOLDEN, f"kitti_{tag}_11.pgm"), out])
    img = _read_ppm(out + "hsbresenhamLineFlow.ppm")  # RGB order in the file
    lab = np.zeros(img.shape[:2], np.uint8)
    lab[(img[..., 0] == 0) & (img[..., 1] == 255) & (img[..., 2] == 0)] = 1
    lab[(img[..., 0] == 255) & (img[..., 1] == 0) & (img[..., 2] == 0)] = 2
    ref, amb = kat_labels(tag)
    assert int(np.count_nonzero((lab != ref) & ~amb)) == 0
    u = _read_fs_matrix(out + "uMatrixHS.txt")
    from conftest import read_pgm
    a = read_pgm(os.path.join(GOLDEN, f"kitti_{tag}_10.pgm"))
    b = read_pgm(os.path.join(GOLDEN, f"kitti_{tag}_11.pgm"))
    uo, _ = _oracle_flow(a, b, 5, 100)
    assert norm_rel_err(u, uo) <= TOL


@pytest.mark.parametrize("kernel", [0, 2, 4])  # automatic, K2 tiles, K4 strips
@pytest.mark.parametrize("batch", [1, 3])
def test_device_solve_captures_into_a_hip_graph(hs, batch, kernel):
    """include/hsflow.h: the *_device calls are stream-ordered and never
    allocate or synchronise, so a whole solve (K1, the K2 passes, the batch
    split over side streams with event fork/join) can be captured into a
    hipGraph and replayed; the replay gives the eager result bit for bit."""
    import torch
    hs.set_jacobi_kernel(kernel)
    try:
        _capture_and_replay(hs, batch)
    finally:
        hs.set_jacobi_kernel(0)


@pytest.mark.parametrize("kernel", [0, 2])
def test_batch_capture_on_a_stream_forked_from_the_origin(hs, kernel):
    """A batch-3 solve captured on a stream B forked from the capture's
    origin A (the library's automatic setting does not split batches under
    capture: on ROCm 7.2 a stream forked from a capturing non-origin stream
    crashes hipStreamEndCapture, profiles/r04_capture_crash.txt); the replay
    equals the eager solve bit for bit."""
    import torch
    assert hs.max_streams() == 0
    hs.set_jacobi_kernel(kernel)
    try:
        batch, rows, cols = 3, 150, 250
        pairs = [hs.synth_pair(1700 + k, rows, cols) for k in range(batch)]
        t0 = torch.stack([torch.from_numpy(p[0]) for p in pairs]).cuda()
        t1 = torch.stack([torch.from_numpy(p[1]) for p in pairs]).cuda()
        u = torch.empty_like(t0)
        v = torch.empty_like(t0)
        ws = hs.alloc_workspace(rows, cols, batch)
        hs.flow_device(t0, t1, 5, 40, 1.0, u, v, ws)  # eager, split over side streams
        torch.cuda.synchronize()
        ref = (u.clone(), v.clone())
        g = torch.cuda.CUDAGraph()
        B = torch.cuda.Stream()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            A = torch.cuda.current_stream()
            B.wait_stream(A)  # B joins the capture: forked from the origin
            with torch.cuda.stream(B):
                hs.flow_device(t0, t1, 5, 40, 1.0, u, v, ws, B)
            A.wait_stream(B)
        u.fill_(float("nan"))
        v.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(u, ref[0]) and torch.equal(v, ref[1])
    finally:
        hs.set_jacobi_kernel(0)


def test_max_streams_setting_round_trips(hs):
    """hsflow_max_streams reports hsflow_set_max_streams; max_streams_as
    restores the caller's setting (row_bands.graphed and the bench use it)."""
    assert hs.max_streams() == 0
    with hs.max_streams_as(3):
        assert hs.max_streams() == 3
        with hs.max_streams_as(1):
            assert hs.max_streams() == 1
        assert hs.max_streams() == 3
    assert hs.max_streams() == 0


def _capture_and_replay(hs, batch):
    import torch
    pairs = [hs.synth_pair(1500 + k, 120, 210) for k in range(batch)]
    t0 = torch.stack([torch.from_numpy(p[0]) for p in pairs]).cuda()
    t1 = torch.stack([torch.from_numpy(p[1]) for p in pairs]).cuda()
    u = torch.empty_like(t0)
    v = torch.empty_like(t0)
    ws = hs.alloc_workspace(120, 210, batch)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        hs.flow_device(t0, t1, 5, 40, 1.0, u, v, ws)   # eager (creates side streams)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    ref = (u.clone(), v.clone())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        hs.flow_device(t0, t1, 5, 40, 1.0, u, v, ws)
    u.zero_()
    v.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(u, ref[0]) and torch.equal(v, ref[1])
    t0.add_(0)  # inputs unchanged; a second replay is identical too
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(u, ref[0])


def test_16k_square_plane_offsets(hs):
    """A 16384 x 16384 pair (1 GiB per f32 plane): 32-bit byte offsets of
    the buffer descriptors stay exact; blocking depth invariance and the
    oracle on a crop solved in place (rows/cols far from the origin)."""
    import torch
    n = 16384
    I0, I1 = hs.synth_pair(1234, n, n)
    t0, t1 = torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()
    a = _device_flow(hs, t0, t1, 5, 12, 6)
    b = _device_flow(hs, t0, t1, 5, 12, 4)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert np.isfinite(a[0]).all() and 0.05 < float(a[0].mean()) < 0.3
    # a crop's interior (24 px from its edges: 12 iterations x 2 px) equals the
    # full-frame solution there
    r0, c0, h, w = n - 300, n - 400, 300, 400
    uo, _ = oracle.flow(I0[r0:, c0:].copy(), I1[r0:, c0:].copy(), 5, 12, 1.0, nthreads=8)
    assert norm_rel_err(a[0][r0 + 24:n - 1, c0 + 24:n - 1], uo[24:h - 1, 24:w - 1]) <= TOL
    del t0, t1
    torch.cuda.empty_cache()


# ------------------------------------------ round 4: wider full-size parity
def test_full_size_alpha5_window4_against_oracle(hs):
    """A full 1080p frame off the defaults: alpha 5 (hornSchunck.cpp:68,
    alpha^2 in the denominator) and the even window 4 (anchor w - w/2 - 1 = 1,
    hornSchunck.cpp:53-54: an asymmetric 4x4 box), 50 iterations, against
    the float64 oracle."""
    import torch
    I0, I1 = hs.synth_pair(1000, 1080, 1920)
    u, v = hs.flow_device(torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda(),
                          4, 50, 5.0)
    uo, vo = oracle.flow(I0, I1, 4, 50, 5.0, nthreads=16)
    eu, ev = norm_rel_err(u.cpu().numpy(), uo), norm_rel_err(v.cpu().numpy(), vo)
    print(f"1080p alpha 5 w 4 x 50: max|du|/max|u| = {eu:.2e}, dv {ev:.2e}")
    assert eu <= TOL and ev <= TOL


# ------------------------------- round 4: the pipelined host-buffer path
@pytest.mark.parametrize("shape", [(1080, 1920), (1081, 1923), (37, 2050), (300, 49)])
def test_host_api_pipelined_io_bits(hs, ctx, shape):
    """hsflow_flow's chunked upload / download (hsflow_hostio.cpp) returns
    the device solve's bits: f64 outputs are the f32 solve widened, f32
    outputs equal it, reused output buffers (the cv::Mat::create path) equal
    fresh ones, and a strided (ROI) input equals its dense copy."""
    import torch
    rows, cols = shape
    I0, I1 = hs.synth_pair(77, rows, cols, dtype=np.uint8)
    ud, vd = hs.flow_device(torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda(), 5, 24, 1.0)
    ud, vd = ud.cpu().numpy(), vd.cpu().numpy()
    u, v = ctx.flow(I0, I1, 5, 24, 1.0)
    assert u.dtype == np.float64
    assert np.array_equal(u, ud.astype(np.float64)) and np.array_equal(v, vd.astype(np.float64))
    u32, v32 = ctx.flow(I0, I1, 5, 24, 1.0, out_dtype=np.float32)
    assert np.array_equal(u32, ud) and np.array_equal(v32, vd)
    ur = np.full((rows, cols), np.nan)
    vr = np.full((rows, cols), np.nan)
    got = hs.hornSchunck(5, 24, 1.0, context=ctx).getFlow(I0, I1, ur, vr)
    assert got[0] is ur and got[1] is vr  # written in place
    assert np.array_equal(ur, u) and np.array_equal(vr, v)
    big0 = np.zeros((rows + 3, cols + 5), np.uint8)
    big1 = np.zeros_like(big0)
    big0[2:2 + rows, 3:3 + cols] = I0
    big1[2:2 + rows, 3:3 + cols] = I1
    ur2, vr2 = ctx.flow(big0[2:2 + rows, 3:3 + cols], big1[2:2 + rows, 3:3 + cols], 5, 24, 1.0)
    assert np.array_equal(ur2, u) and np.array_equal(vr2, v)


def test_host_api_concurrent_contexts(hs):
    """Several host threads, each with its own context, call hsflow_flow at
    once (the copy pool serves one of them, the others copy inline): every
    result equals the same pair solved alone."""
    import threading
    pairs = [hs.synth_pair(500 + k, 540, 960, dtype=np.uint8) for k in range(4)]
    ref = []
    with hs.Context(0) as c0:
        for I0, I1 in pairs:
            ref.append(c0.flow(I0, I1, 5, 30, 1.0))
    out = [None] * len(pairs)
    errs = []

    def run(k):
        try:
            with hs.Context(0) as c:
                for _ in range(3):
                    out[k] = c.flow(pairs[k][0], pairs[k][1], 5, 30, 1.0)
        except Exception as e:  # pragma: no cover
            errs.append(repr(e))

    ts = [threading.Thread(target=run, args=(k,)) for k in range(len(pairs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errs, errs
    for k in range(len(pairs)):
        assert np.array_equal(out[k][0], ref[k][0]) and np.array_equal(out[k][1], ref[k][1])


def test_flow_multi_release_and_reuse(hs, ctx):
    """hsflow_flow_multi_release drops the kept per-device contexts; the next
    multi call builds them again and gives the same bits."""
    pairs = [hs.synth_pair(900 + k, 200, 310, dtype=np.uint8) for k in range(3)]
    a = hs.flow_multi([0, 0], pairs, 5, 20, 1.0)
    hs.flow_multi_release()
    b = hs.flow_multi([0], pairs, 5, 20, 1.0)
    for (ua, va), (ub, vb), (I0, I1) in zip(a, b, pairs):
        uc, vc = ctx.flow(I0, I1, 5, 20, 1.0)
        assert np.array_equal(ua, ub) and np.array_equal(va, vb)
        assert np.array_equal(ua, uc) and np.array_equal(va, vc)
