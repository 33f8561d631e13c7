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
