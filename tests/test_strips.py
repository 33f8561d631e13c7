"""K4, the streaming-strip Jacobi pass (csrc/hsflow_strips.hip), against K2's
register tiles and the float64 oracle.

K4 adds the window sums in K2's order (horizontal association by column
parity, vertical by image-row parity), so the two kernels must give the same
bits for every shape, blocking depth, segment height, pass direction and
gradient format; the oracle bounds both at 1e-4 (north_star).  The
host-side plan (which kernel, which segment height) is checked without a
GPU in test_abi.py."""
import numpy as np
import pytest
import torch

from conftest import norm_rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-4


def _pairs(hs, batch, rows, cols, nonint=(), seed=1000):
    ps = [hs.synth_pair(seed + i, rows, cols) for i in range(batch)]
    I0 = np.stack([p[0] for p in ps])
    I1 = np.stack([p[1] for p in ps])
    for i in nonint:  # non-integral frames: the f32-gradient planes
        I0[i] = I0[i] + 0.375
    return torch.from_numpy(I0).cuda(), torch.from_numpy(I1).cuda()


def _solve(hs, kernel, I0, I1, w, iters, seg_rows=0, warm=None):
    hs.set_jacobi_kernel(kernel)
    hs.set_strip_rows(seg_rows)
    try:
        if warm is None:
            u, v = hs.flow_device(I0, I1, w, iters, 1.0)
        else:
            rows, cols = I0.shape[-2:]
            ws = hs.alloc_workspace(rows, cols, I0.shape[0])
            hs.gradients_device(I0, I1, ws)
            u, v = warm[0].clone(), warm[1].clone()
            hs.jacobi_device(rows, cols, I0.shape[0], w, iters, 1.0, u, v, ws, warm_start=True)
        torch.cuda.synchronize()
        return u, v
    finally:
        hs.set_jacobi_kernel(0)
        hs.set_strip_rows(0)


@pytest.mark.parametrize("batch,rows,cols,w,iters", [
    (1, 1, 1, 5, 12), (1, 2, 3, 5, 7), (2, 37, 53, 5, 13), (1, 300, 49, 3, 17),
    (3, 64, 130, 5, 12), (2, 101, 333, 3, 24), (1, 375, 1242, 5, 100),
    (1, 375, 1242, 3, 100), (2, 200, 257, 5, 30), (1, 90, 256, 5, 6),
    (2, 1080, 1920, 5, 18), (1, 2160, 3840, 3, 16),
])
def test_k4_bits_equal_k2(hs, batch, rows, cols, w, iters):
    """Forced K4 vs forced K2: odd widths (dword path), 1x1 and ragged
    planes, a shorter last pass
    (K2), every window K4 is built for."""
    I0, I1 = _pairs(hs, batch, rows, cols)
    a = _solve(hs, 2, I0, I1, w, iters)
    b = _solve(hs, 4, I0, I1, w, iters)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("kb", [4, 5])
@pytest.mark.parametrize("batch,rows,cols,iters,seg_rows", [
    (1, 2, 3, 11, 0), (2, 37, 53, 13, 0), (1, 375, 1242, 100, 0), (2, 200, 257, 30, 16),
    (1, 1080, 1920, 42, 40), (1, 2160, 3840, 20, 32), (3, 64, 131, 17, 24),
])
def test_k4_shallow_depths_bits_equal_k2(hs, kb, batch, rows, cols, iters, seg_rows):
    """K4 built at KB 4 and 5 for w = 5 (fewer registers per wave: more
    waves per SIMD for launches that fill part of the chip) gives K2's bits
    too: odd widths, 1-row-ish planes, short segments, a shorter last pass."""
    I0, I1 = _pairs(hs, batch, rows, cols)
    hs.set_iters_per_launch(kb)
    try:
        a = _solve(hs, 2, I0, I1, 5, iters)
        b = _solve(hs, 4, I0, I1, 5, iters, seg_rows=seg_rows)
    finally:
        hs.set_iters_per_launch(0)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("seg_rows", [12, 36, 84, 240])
def test_k4_segment_height_invariance(hs, seg_rows):
    I0, I1 = _pairs(hs, 2, 257, 390)
    ref = _solve(hs, 2, I0, I1, 5, 24)
    got = _solve(hs, 4, I0, I1, 5, 24, seg_rows=seg_rows)
    assert torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1])


@pytest.mark.parametrize("w", [3, 5])
def test_k4_warm_start_and_mixed_gradient_formats(hs, w):
    """A batch mixing integral (packed gradients) and non-integral (f32
    planes) pairs, continued from a random warm start."""
    I0, I1 = _pairs(hs, 3, 120, 200, nonint=(1,))
    g = torch.Generator(device="cuda").manual_seed(7)
    warm = (torch.randn(3, 120, 200, device="cuda", generator=g),
            torch.randn(3, 120, 200, device="cuda", generator=g))
    a = _solve(hs, 2, I0, I1, w, 24, warm=warm)
    b = _solve(hs, 4, I0, I1, w, 24, warm=warm)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("w", [3, 5])
def test_k4_against_the_oracle(hs, w):
    import oracle
    a, b = hs.synth_pair(1234, 180, 260)
    I0, I1 = torch.from_numpy(a)[None].cuda(), torch.from_numpy(b)[None].cuda()
    u, v = _solve(hs, 4, I0, I1, w, 60)
    uo, vo = oracle.flow(a, b, w, 60, 1.0)
    assert norm_rel_err(u[0].cpu().numpy(), uo) <= TOL
    assert norm_rel_err(v[0].cpu().numpy(), vo) <= TOL


def test_automatic_choice_runs_k4_on_the_bench_shapes(hs):
    assert hs.jacobi_kernel_name(1080, 1920, 8, 5) == "hs_jacobi_strip_kernel"
    assert hs.jacobi_kernel_name(2160, 3840, 2, 5) == "hs_jacobi_strip_kernel"
    assert hs.jacobi_kernel_name(1080, 1920, 8, 3) == "hs_jacobi_strip_kernel"


def test_non_integral_float64_frames_against_the_oracle(hs):
    """CV_64FC1 frames with non-integral values (the reference converts with
    convertTo(CV_64FC1) and takes Sobel in float64, hornSchunck.cpp:23-28):
    the host API uploads them as float64 and K1 sums in float64, each
    gradient rounded to f32 once; u, v within 1e-4 of the float64 oracle."""
    import oracle
    rng = np.random.default_rng(5)
    a, b = hs.synth_pair(1300, 150, 210)
    I0 = a.astype(np.float64) + rng.uniform(-0.5, 0.5, a.shape) + 1e-3 * np.pi
    I1 = b.astype(np.float64) + rng.uniform(-0.5, 0.5, b.shape)
    u, v = hs.hornSchunck(5, 80, 1.0).getFlow(I0, I1)
    uo, vo = oracle.flow(I0, I1, 5, 80, 1.0)
    assert u.dtype == np.float64
    assert norm_rel_err(u, uo) <= TOL and norm_rel_err(v, vo) <= TOL
    # the gradients themselves: f64 sums rounded once to f32 (half an f32
    # ulp from the oracle's f64 values, up to its own summation order)
    gx, gy, gt = hs.hornSchunck(5, 80, 1.0).getGradients(I0, I1)
    gxo, gyo, gto = oracle.gradients(I0, I1)
    for got, ref in ((gx, gxo), (gy, gyo), (gt, gto)):
        assert np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1e-3)) <= 1.2e-7


def test_float64_device_tensors(hs):
    a, b = hs.synth_pair(1301, 96, 160)
    t0 = torch.from_numpy(a.astype(np.float64))[None].cuda()
    t1 = torch.from_numpy(b.astype(np.float64))[None].cuda()
    u64, v64 = hs.flow_device(t0, t1, 5, 30, 1.0)
    u32, v32 = hs.flow_device(t0.float(), t1.float(), 5, 30, 1.0)
    torch.cuda.synchronize()
    assert torch.equal(u64, u32) and torch.equal(v64, v32)  # integral frames: same bits


@pytest.mark.parametrize("cols", [4096, 4097])
def test_k4_bits_equal_k2_at_the_plane_size_cap(hs, cols):
    """A plane within a few rows of the 2^29-pixel cap (2 GiB of f32 per
    plane): K4 streams up to KB AR + D rows past the bottom edge, whose byte
    offsets pass 2^31; those rows must still read as zero in every lane
    (also the lanes outside the image columns), so K4 keeps K2's bits down
    to the last row.  Random u8 frames made on the device; one 6-iteration
    pass."""
    rows = ((1 << 29) - 1) // cols
    g = torch.Generator(device="cuda")
    g.manual_seed(4)
    I0 = torch.randint(0, 256, (1, rows, cols), dtype=torch.uint8, device="cuda", generator=g)
    I1 = torch.randint(0, 256, (1, rows, cols), dtype=torch.uint8, device="cuda", generator=g)
    a = _solve(hs, 2, I0, I1, 5, 6)
    b = _solve(hs, 4, I0, I1, 5, 6)
    for x, y in zip(a, b):
        assert torch.equal(x[0, -256:], y[0, -256:]), "bottom rows differ"
        assert torch.equal(x, y)
        assert bool(torch.isfinite(y[0, -256:]).all())
    del a, b, I0, I1
    torch.cuda.empty_cache()
