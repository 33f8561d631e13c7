"""Frame sources and the streaming front-end (cpp-optical-flow_amd/frames.py,
SURVEY §8f item 4): the reference's input stage main.cpp:48-64 (imread of
two files, or two frames of a video by index) over the decoder-free
containers of this image, feeding the frame-parallel driver.

The luma->gray rule for YUV4MPEG2 is not pinned by any reference artefact
(no decoder exists here); it is tested against its own definition."""
import os
import subprocess

import numpy as np
import pytest

import frames as fr
from conftest import GOLDEN, ROOT, read_pgm


def _bgr_frames(n, rows, cols, seed=5):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (rows + 4 * n, cols + 4 * n, 3), dtype=np.uint8)
    return [np.ascontiguousarray(base[2 * k:2 * k + rows, 3 * k:3 * k + cols]) for k in range(n)]


# ----------------------------------------------------------------- CPU
def test_pnm_round_trip_and_rgb_order(tmp_path):
    bgr = _bgr_frames(1, 9, 13)[0]
    p = str(tmp_path / "a.ppm")
    fr.write_pnm(p, bgr)
    assert np.array_equal(fr.read_pnm(p), bgr)
    raw = open(p, "rb").read()
    assert raw[-3:] == bytes(bgr[-1, -1, ::-1])        # file holds RGB, imread gives BGR
    g = bgr[..., 0]
    fr.write_pnm(str(tmp_path / "g.pgm"), g)
    assert np.array_equal(fr.read_pnm(str(tmp_path / "g.pgm")), g)


def test_pnm_reads_the_reference_gray_fixtures():
    a = fr.read_pnm(os.path.join(GOLDEN, "kitti_000050_10.pgm"))
    assert np.array_equal(a, read_pgm(os.path.join(GOLDEN, "kitti_000050_10.pgm")))


def test_image_sequence_seek_and_errors(tmp_path):
    frames = _bgr_frames(4, 8, 10)
    paths = []
    for k, f in enumerate(frames):
        paths.append(str(tmp_path / f"{k:04d}.ppm"))
        fr.write_pnm(paths[-1], f)
    src = fr.open_source(str(tmp_path))
    assert len(src) == 4
    for k in (3, 0, 2):
        assert np.array_equal(src.read(k), frames[k])
    with pytest.raises(fr.FrameError):
        src.read(4)


def test_image_sequence_png_through_pillow(tmp_path):
    PIL = pytest.importorskip("PIL.Image")
    bgr = _bgr_frames(1, 7, 11)[0]
    p = str(tmp_path / "x.png")
    PIL.fromarray(np.ascontiguousarray(bgr[:, :, ::-1])).save(p)
    assert np.array_equal(fr.ImageSequence([p]).read(0), bgr)


def test_raw_video_seek(tmp_path):
    frames = _bgr_frames(5, 6, 9)
    p = str(tmp_path / "v.bgr24")
    with open(p, "wb") as f:
        for x in frames:
            f.write(x.tobytes())
        f.write(b"\x01\x02")                       # trailing partial frame ignored
    src = fr.open_source(p, 6, 9)
    assert len(src) == 5
    for k in (4, 1, 1, 0):
        assert np.array_equal(src.read(k), frames[k])
    with pytest.raises(fr.FrameError):
        src.read(5)


def test_y4m_mono_full_and_video_range(tmp_path):
    g = [np.full((4, 6), v, np.uint8) for v in (0, 16, 17, 126, 235, 255)]
    p = str(tmp_path / "full.y4m")
    fr.write_y4m(p, g, full_range=True)
    src = fr.Y4MVideo(p)
    assert len(src) == 6 and all(np.array_equal(src.read(k), g[k]) for k in range(6))
    p2 = str(tmp_path / "video.y4m")
    fr.write_y4m(p2, g, full_range=False)
    src2 = fr.Y4MVideo(p2)
    exp = [0, 0, 1, 128, 255, 255]   # round((Y - 16) * 255 / 219), clamped
    for k, e in enumerate(exp):
        assert int(src2.read(k)[0, 0]) == e
    y = np.arange(256)
    ref = np.clip(np.floor((y - 16) * 255 / 219 + 0.5), 0, 255)
    got = np.clip(np.floor_divide((y - 16) * 255 + 109, 219), 0, 255)
    assert np.array_equal(ref, got)


def test_y4m_420_with_frame_parameters(tmp_path):
    rows, cols = 5, 7
    lum = [np.arange(rows * cols, dtype=np.uint8).reshape(rows, cols) + k for k in range(3)]
    chroma = 2 * ((cols + 1) // 2) * ((rows + 1) // 2)
    p = str(tmp_path / "c420.y4m")
    with open(p, "wb") as f:
        f.write(b"YUV4MPEG2 W7 H5 F30:1 C420jpeg XCOLORRANGE=FULL\n")
        for k, y in enumerate(lum):
            f.write(b"FRAME Ixyz\n" if k == 1 else b"FRAME\n")
            f.write(y.tobytes() + bytes([128]) * chroma)
    src = fr.open_source(p)
    assert len(src) == 3
    assert np.array_equal(src.read(2), lum[2]) and np.array_equal(src.read(1), lum[1])


@pytest.mark.parametrize("tag", [b"C420p10", b"C444p12", b"Cmono16", b"C422p10",
                                 b"C444alpha"])
def test_y4m_rejects_high_bit_depth_and_alpha(tmp_path, tag):
    p = str(tmp_path / "hbd.y4m")
    with open(p, "wb") as f:
        f.write(b"YUV4MPEG2 W4 H2 F25:1 " + tag + b"\nFRAME\n" + bytes(64))
    with pytest.raises(fr.FrameError, match="unsupported"):
        fr.open_source(p)


def test_capture_pair_and_consecutive_pairs(tmp_path):
    a = fr.ImageSequence([])
    with pytest.raises(fr.FrameError):
        fr.capture_pair(a, 0, 1)
    frames = _bgr_frames(3, 6, 8)
    p = str(tmp_path / "v.bgr24")
    with open(p, "wb") as f:
        for x in frames:
            f.write(x.tobytes())
    src = fr.RawVideo(p, 6, 8)
    x, y = fr.capture_pair(src, 2, 0)                 # main.cpp:53-59 seeks by index
    assert np.array_equal(x, frames[2]) and np.array_equal(y, frames[0])
    assert fr.consecutive_pairs(5) == [(0, 1), (1, 2), (2, 3), (3, 4)]
    assert fr.consecutive_pairs(5, start=1, count=2, gap=2) == [(1, 3), (2, 4)]


def test_pair_windows():
    pairs = fr.consecutive_pairs(20)
    w = fr.pair_windows(pairs, 8)
    assert [len(x) for x in w] == [8, 8, 3]
    assert sum(w, []) == list(range(19))
    assert fr.pair_windows([], 8) == []


# ----------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_stream_of_bgr_frames_equals_per_pair_solves(tmp_path):
    import torch
    import hsflow
    frames = _bgr_frames(5, 90, 130)
    p = str(tmp_path / "v.bgr24")
    with open(p, "wb") as f:
        for x in frames:
            f.write(x.tobytes())
    src = fr.RawVideo(p, 90, 130)
    pairs = fr.consecutive_pairs(len(src))
    out = fr.solve_stream(src, pairs, 5, 30, 1.0)
    torch.cuda.synchronize()
    ctx = hsflow.Context(0)
    for (a, b), (u, v) in zip(pairs, out):
        ur, vr = ctx.flow_bgr(frames[a], frames[b], 5, 30, 1.0, out_dtype=np.float32)
        assert np.array_equal(u.cpu().numpy(), ur) and np.array_equal(v.cpu().numpy(), vr)
    ctx.close()


@pytest.mark.gpu
def test_y4m_stream_and_cpp_driver(tmp_path):
    """The Python stream and examples/hs_main's video branch (main.cpp:53-59
    over .y4m) give the flow of the same gray frames."""
    import torch
    import hsflow
    a = read_pgm(os.path.join(GOLDEN, "kitti_000050_10.pgm"))[:96, :160]
    b = read_pgm(os.path.join(GOLDEN, "kitti_000050_11.pgm"))[:96, :160]
    p = str(tmp_path / "k.y4m")
    fr.write_y4m(p, [a, b, a], full_range=True)
    src = fr.Y4MVideo(p)
    (u, v), = fr.solve_stream(src, [(0, 1)], 5, 100, 1.0)
    ctx = hsflow.Context(0)
    ur, vr = ctx.flow(a, b, 5, 100, 1.0, out_dtype=np.float32)
    ctx.close()
    assert np.array_equal(u.cpu().numpy(), ur) and np.array_equal(v.cpu().numpy(), vr)
    exe = os.path.join(ROOT, "examples", "hs_main")
    out = str(tmp_path / "r_")
    subprocess.check_call([exe, p, "0", "1", out])
    txt = open(out + "uMatrixHS.txt").read()
    body = txt.split("data: [")[1].split("]")[0]
    uc = np.array([float(x) for x in body.replace("\n", " ").split(",")]).reshape(96, 160)
    assert np.array_equal(uc, ur.astype(np.float64))
    with pytest.raises(subprocess.CalledProcessError):
        subprocess.check_call([exe, p, "0", "7", out])   # frame 7 does not exist -> -1


class _CountingSource:
    """A source that counts its reads (solve_stream reads each frame once)."""

    def __init__(self, frames):
        self.frames, self.reads = frames, []

    def __len__(self):
        return len(self.frames)

    def read(self, i):
        self.reads.append(i)
        return self.frames[i]


@pytest.mark.gpu
def test_kitti_y4m_stream_against_the_float64_oracle(tmp_path):
    """main.cpp:53-59 over a video: the KITTI 000050 pair (the reference's
    own frames, 15-bit gray fixtures) as a YUV4MPEG2 stream of 2 x 9 frames
    (a, b, a, b, ...), every consecutive pair solved by solve_stream in
    batched windows (8 pairs per batch: two windows, the second a partial
    one) -- each (u, v) within the north_star tolerance (1e-4, norm-relative)
    of the float64 oracle's restatement of hornSchunck.cpp, not of hsflow
    itself; each frame read once."""
    import torch
    import oracle
    from conftest import norm_rel_err
    a = read_pgm(os.path.join(GOLDEN, "kitti_000050_10.pgm"))
    b = read_pgm(os.path.join(GOLDEN, "kitti_000050_11.pgm"))
    p = str(tmp_path / "kitti.y4m")
    seq = [a, b] * 9
    fr.write_y4m(p, seq, full_range=True)
    src = _CountingSource([fr.Y4MVideo(p).read(i) for i in range(len(seq))])
    pairs = fr.consecutive_pairs(len(src))
    out = fr.solve_stream(src, pairs, 5, 100, 1.0, batch=8)
    torch.cuda.synchronize()
    assert len(out) == len(pairs) == 17
    assert sorted(src.reads) == list(range(18))             # lazy: each frame once
    ab = oracle.flow(a.astype(np.float64), b.astype(np.float64), 5, 100, 1.0)
    ba = oracle.flow(b.astype(np.float64), a.astype(np.float64), 5, 100, 1.0)
    for k, (u, v) in enumerate(out):
        uo, vo = ab if k % 2 == 0 else ba
        assert norm_rel_err(u.cpu().numpy(), uo) <= 1e-4, k
        assert norm_rel_err(v.cpu().numpy(), vo) <= 1e-4, k
    # the flow checksum of this pair (the float64 restatement
    # that reproduces the reference's arrow plot pixel-exactly)
    assert abs(float(ab[0].sum()) - (-9517.890763654887)) < 1e-6
    assert abs(float(out[0][0].double().sum()) - float(ab[0].sum())) < 0.05
    # on_flow: the flows handed over window by window, nothing kept
    got = {}
    assert fr.solve_stream(src, pairs[:10], 5, 100, 1.0, batch=4,
                           on_flow=lambda k, u, v: got.__setitem__(k, u.clone())) is None
    assert sorted(got) == list(range(10))
    for k in range(10):
        assert torch.equal(got[k], out[k][0])
