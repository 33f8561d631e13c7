"""K3 (streaming strips, csrc/hsflow_stream.hip) against K2 (register tiles)
and the float64 oracle.

K3 runs the same per-pixel operation sequence as K2 (hsflow_device.h), so
every case is checked BIT-EXACTLY against K2 (np.array_equal), and a few
against the oracle at the parity bar max|d| / max|ref| <= 1e-4.  Cases cover
the pieces K3 adds: segment boundaries (many short segments on small batches,
one whole-strip segment on large ones), rows fewer than the pipeline depth,
strips at the image's right edge, non-integral frames (f32 gradient planes),
mixed batches, warm starts, partial last passes (K2 takes them) and odd widths
(K2 throughout).
"""
import numpy as np
import pytest

import oracle
from conftest import norm_rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-4


@pytest.fixture(scope="module")
def hs():
    import hsflow
    yield hsflow
    hsflow.set_jacobi_kernel(0)


def _solve(hs, kernel, t0, t1, w, n, u=None, v=None):
    import torch
    hs.set_jacobi_kernel(kernel)
    try:
        if u is None:
            uu, vv = hs.flow_device(t0, t1, w, n, 1.0)
        else:
            import ctypes
            uu, vv = u.clone(), v.clone()
            rows, cols = t0.shape[-2:]
            batch = int(np.prod(t0.shape[:-2])) if t0.dim() > 2 else 1
            ws = hs.alloc_workspace(rows, cols, batch, t0.device)
            rc = hs.lib().hsflow_gradients_device(
                t0.data_ptr(), t1.data_ptr(), hs._tensor_dtype(t0), rows, cols, batch,
                None, None, None, ws.data_ptr(), ws.numel(), None)
            assert rc == 0
            rc = hs.lib().hsflow_jacobi_device(rows, cols, batch, w, n, ctypes.c_float(1.0),
                                               1, uu.data_ptr(), vv.data_ptr(), ws.data_ptr(),
                                               ws.numel(), None)
            assert rc == 0
        torch.cuda.synchronize()
    finally:
        hs.set_jacobi_kernel(0)
    return uu.cpu().numpy(), vv.cpu().numpy()


def _pair(hs, seed, rows, cols, batch=1, dtype=np.float32, shift=0.0):
    import torch
    I0s, I1s = [], []
    for b in range(batch):
        I0, I1 = hs.synth_pair(seed + b, rows, cols)
        I0s.append(I0.astype(np.float32) + np.float32(shift))
        I1s.append(I1.astype(np.float32))
    I0 = np.stack(I0s) if batch > 1 else I0s[0]
    I1 = np.stack(I1s) if batch > 1 else I1s[0]
    t0 = torch.from_numpy(I0.astype(dtype)).cuda()
    t1 = torch.from_numpy(I1.astype(dtype)).cuda()
    return I0, I1, t0, t1


def _same(a, b):
    return np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.mark.parametrize("w,n", [(5, 6), (5, 12), (5, 23), (3, 8), (3, 19)])
@pytest.mark.parametrize("shape", [(300, 518), (64, 128), (17, 130), (5, 2), (1, 2),
                                   (131, 210)])
def test_k3_equals_k2(hs, w, n, shape):
    rows, cols = shape
    _, _, t0, t1 = _pair(hs, 11, rows, cols)
    assert _same(_solve(hs, 3, t0, t1, w, n), _solve(hs, 2, t0, t1, w, n))


@pytest.mark.parametrize("dtype", [np.uint8, np.float16])
def test_k3_input_dtypes(hs, dtype):
    _, _, t0, t1 = _pair(hs, 5, 150, 260, batch=2, dtype=dtype)
    assert _same(_solve(hs, 3, t0, t1, 5, 18), _solve(hs, 2, t0, t1, 5, 18))


def test_k3_non_integral_frames_use_f32_gradients(hs):
    I0, I1, t0, t1 = _pair(hs, 8, 120, 334, shift=0.3)
    got = _solve(hs, 3, t0, t1, 5, 12)
    assert _same(got, _solve(hs, 2, t0, t1, 5, 12))
    uo, vo = oracle.flow(I0, I1, 5, 12, 1.0, nthreads=8)
    assert norm_rel_err(got[0], uo) <= TOL and norm_rel_err(got[1], vo) <= TOL


def test_k3_mixed_batch(hs):
    """One integral and one non-integral pair in one launch."""
    import torch
    _, _, a0, a1 = _pair(hs, 21, 96, 202)
    _, _, b0, b1 = _pair(hs, 22, 96, 202, shift=0.5)
    t0 = torch.stack([a0, b0])
    t1 = torch.stack([a1, b1])
    assert _same(_solve(hs, 3, t0, t1, 5, 12), _solve(hs, 2, t0, t1, 5, 12))


def test_k3_warm_start(hs):
    import torch
    _, _, t0, t1 = _pair(hs, 31, 140, 300)
    g = torch.Generator().manual_seed(3)
    u = torch.randn((140, 300), generator=g).cuda()
    v = torch.randn((140, 300), generator=g).cuda()
    assert _same(_solve(hs, 3, t0, t1, 5, 12, u, v), _solve(hs, 2, t0, t1, 5, 12, u, v))


def test_k3_large_batch_whole_strip_segments(hs):
    """Enough strips to fill the GPU: one segment per strip (seg = rows)."""
    _, _, t0, t1 = _pair(hs, 40, 70, 2080, batch=80)
    assert _same(_solve(hs, 3, t0, t1, 5, 6), _solve(hs, 2, t0, t1, 5, 6))


def test_k3_odd_width_falls_back(hs):
    _, _, t0, t1 = _pair(hs, 41, 90, 333)
    assert _same(_solve(hs, 3, t0, t1, 5, 12), _solve(hs, 2, t0, t1, 5, 12))


def test_k3_1080p_against_oracle(hs):
    I0, I1, t0, t1 = _pair(hs, 1000, 1080, 1920)
    got = _solve(hs, 3, t0, t1, 5, 30)
    assert _same(got, _solve(hs, 2, t0, t1, 5, 30))
    uo, vo = oracle.flow(I0, I1, 5, 30, 1.0, nthreads=8)
    assert norm_rel_err(got[0], uo) <= TOL and norm_rel_err(got[1], vo) <= TOL
