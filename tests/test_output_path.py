"""GPU output path: hsflow_download_device, the stream-ordered device ->
pinned-host download bench.py's end-to-end leg uses for u, v (main.cpp:98-107
consume the flow on the host).  Byte work, so checked bit-exactly."""
import pytest


@pytest.fixture(scope="module")
def hs():
    import hsflow
    return hsflow


@pytest.mark.gpu
@pytest.mark.parametrize("nbytes", [1, 4, 7679, 7680, 3 * 7680 + 5, 1920 * 1080 * 4,
                                    2 * 3840 * 2160 * 4 + 12])
def test_download_device_is_bit_exact(hs, nbytes):
    import torch
    g = torch.Generator().manual_seed(nbytes)
    src_h = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, generator=g)
    src = src_h.cuda()
    dst = torch.full((nbytes,), 7, dtype=torch.uint8).pin_memory()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    hs.download_device(dst, src, s)
    s.synchronize()
    assert torch.equal(dst, src_h)


@pytest.mark.gpu
def test_download_device_is_stream_ordered(hs):
    """The download sees every write queued before it on its stream."""
    import torch
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        src = torch.zeros(1080, 1920, device="cuda")
        src.add_(3.5)
    dst = torch.empty(1080, 1920).pin_memory()
    hs.download_device(dst, src, s)
    s.synchronize()
    assert bool((dst == 3.5).all())


@pytest.mark.gpu
def test_download_device_rejects_mismatched_sizes(hs):
    import torch
    with pytest.raises(hs.HsflowError):
        hs.download_device(torch.empty(8).pin_memory(), torch.empty(9, device="cuda"))


@pytest.mark.gpu
def test_host_call_context_reuse_is_bit_exact(hs):
    """One context through a frame loop (main.cpp:97-98): repeated calls
    reuse its grow-only device buffers and must give a fresh context's bits
    across new frames, new parameters (alpha, iterations, window), a larger
    frame and back, f32 frames and a launch override."""
    import numpy as np
    a, b = hs.synth_pair(7, 270, 480)
    a8, b8 = a.astype(np.uint8), b.astype(np.uint8)
    c, d = hs.synth_pair(8, 270, 480)
    c8, d8 = c.astype(np.uint8), d.astype(np.uint8)
    big0, big1 = (x.astype(np.uint8) for x in hs.synth_pair(9, 540, 960))

    def fresh(I0, I1, w, n, alpha):
        with hs.Context(0) as ctx:  # one call per context: always eager
            return ctx.flow(I0, I1, w, n, alpha)

    ref = fresh(a8, b8, 5, 40, 1.0)
    with hs.Context(0) as ctx:
        for _ in range(4):
            u, v = ctx.flow(a8, b8, 5, 40, 1.0)
            assert np.array_equal(u, ref[0]) and np.array_equal(v, ref[1])
        # new frames, same buffers and parameters
        ref_cd = fresh(c8, d8, 5, 40, 1.0)
        for _ in range(3):
            u, v = ctx.flow(c8, d8, 5, 40, 1.0)
            assert np.array_equal(u, ref_cd[0]) and np.array_equal(v, ref_cd[1])
        # parameters change: alpha, iterations, window
        for args in ((5, 40, 3.0), (5, 41, 3.0), (3, 41, 3.0)):
            want = fresh(a8, b8, *args)
            for _ in range(3):
                u, v = ctx.flow(a8, b8, *args)
                assert np.array_equal(u, want[0]) and np.array_equal(v, want[1]), args
        # a larger frame grows the device buffers, then back to the small one
        want_big = fresh(big0, big1, 5, 40, 1.0)
        for _ in range(3):
            u, v = ctx.flow(big0, big1, 5, 40, 1.0)
            assert np.array_equal(u, want_big[0]) and np.array_equal(v, want_big[1])
        for _ in range(3):
            u, v = ctx.flow(a8, b8, 5, 40, 1.0)
            assert np.array_equal(u, ref[0]) and np.array_equal(v, ref[1])
        # f32 frames take the f32-gradient variant as well
        want_f = fresh(a, b, 5, 40, 1.0)
        for _ in range(3):
            u, v = ctx.flow(a, b, 5, 40, 1.0)
            assert np.array_equal(u, want_f[0]) and np.array_equal(v, want_f[1])
        # a launch override between two identical calls is part of the key
        try:
            hs.set_jacobi_kernel(2)
            for _ in range(3):
                u, v = ctx.flow(a8, b8, 5, 40, 1.0)
                assert np.array_equal(u, ref[0]) and np.array_equal(v, ref[1])
        finally:
            hs.set_jacobi_kernel(0)


@pytest.mark.gpu
@pytest.mark.parametrize("rows,cols,pad", [(1080, 1920, 64), (270, 480, 3), (2160, 3840, 256)])
def test_host_call_into_fresh_roi_outputs(hs, rows, cols, pad):
    """main.cpp:93's fresh `cv::Mat u, v;` -- here as ROIs of larger, freshly
    mapped private buffers (row step > cols x 8 B): the call faults the
    output pages in on its copy threads (huge-page advice, one write per
    page inside the rows) while the solve runs.  The rows get the contiguous
    call's bits and not one byte between or after them changes."""
    import mmap
    import numpy as np
    a, b = hs.synth_pair(11, rows, cols)
    a8, b8 = a.astype(np.uint8), b.astype(np.uint8)
    ctx = hs.Context(0)
    ru, rv = ctx.flow(a8, b8, 5, 24, 1.0)
    step_elems = cols + pad
    planes, maps = [], []
    for _ in range(2):
        m = mmap.mmap(-1, (rows + 1) * step_elems * 8, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        big = np.frombuffer(m, np.float64).reshape(rows + 1, step_elems)
        big[-1, :] = -7.0          # the row after the ROI
        big[:-1, cols:] = -7.0     # the gaps between ROI rows
        maps.append(m)
        planes.append(big)
    u, v = planes[0][:-1, :cols], planes[1][:-1, :cols]
    rc = hs.lib().hsflow_flow(ctx._p, a8.ctypes.data, b8.ctypes.data, hs.U8, rows, cols,
                              a8.strides[0], b8.strides[0], 5, 24, 1.0, u.ctypes.data,
                              v.ctypes.data, hs.F64, u.strides[0])
    hs._check(rc, ctx._p)
    assert np.array_equal(u, ru) and np.array_equal(v, rv)
    for plane in planes:
        assert bool((plane[:-1, cols:] == -7.0).all()) and bool((plane[-1, :] == -7.0).all())
    del u, v, planes, plane, big
    for m in maps:
        m.close()
