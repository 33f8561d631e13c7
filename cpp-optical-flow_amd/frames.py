"""Frame sources: the reference's input stage (HornSchunckOF/main.cpp:48-64)
as a streaming front-end for the frame-parallel driver.

main.cpp reads either two image files (`cv::imread`, :50-51) or two frames
of an .mp4 by index (`cv::VideoCapture`, `capture.set(1, n)` =
CAP_PROP_POS_FRAMES then `capture >> frame`, :53-59), converts both to gray
(:13-14) and solves.  This image has no video decoder (no OpenCV, ffmpeg or
PyAV), so the seekable sources here are the containers that need none:

  ImageSequence  one file per frame: PGM/PPM natively, other formats
                 through Pillow when it is importable (as imread would)
  RawVideo       headerless frames of rows x cols BGR24 (or gray8), memory-
                 mapped: O(1) seek
  Y4MVideo       YUV4MPEG2 (the raw form ffmpeg writes with `-f yuv4mpegpipe`),
                 any chroma layout; frames are indexed once, O(1) seek.  Its
                 gray is the luma plane, expanded from video range (16..235)
                 to 0..255 unless the header says full range -- an
                 approximation of decode-to-BGR + cvtColor that no reference
                 artefact pins (documented as unpinned)

`read(i)` returns BGR uint8 (H x W x 3) or gray (H x W) like imread would;
`capture_pair(src, prev, next)` is main.cpp:53-59; `solve_stream` feeds
consecutive pairs to frame_parallel.run_stream with the BGR->gray
conversion on the GPU (hsflow_bgr_to_gray_device) and libhsflow as solver.
"""
from __future__ import annotations

import os
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np


class FrameError(IOError):
    """A frame that cannot be read (main.cpp:65-68 "Can't read the images")."""


# ------------------------------------------------------------------ sources
def read_pnm(path: str) -> np.ndarray:
    """8-bit PGM (gray) / PPM (returned as BGR, like imread)."""
    with open(path, "rb") as f:
        data = f.read()
    toks, pos = [], 0
    while len(toks) < 4:
        while pos < len(data) and data[pos:pos + 1].isspace():
            pos += 1
        if data[pos:pos + 1] == b"#":
            pos = data.index(b"\n", pos) + 1
            continue
        end = pos
        while end < len(data) and not data[end:end + 1].isspace():
            end += 1
        toks.append(data[pos:end])
        pos = end
    magic, w, h, mx = toks[0], int(toks[1]), int(toks[2]), int(toks[3])
    pos += 1
    if magic not in (b"P5", b"P6") or mx != 255:
        raise FrameError(f"{path}: unsupported PNM ({magic!r}, max {mx})")
    ch = 1 if magic == b"P5" else 3
    px = np.frombuffer(data, np.uint8, count=w * h * ch, offset=pos)
    if ch == 1:
        return px.reshape(h, w).copy()
    return px.reshape(h, w, 3)[:, :, ::-1].copy()  # RGB -> BGR


def write_pnm(path: str, img: np.ndarray) -> None:
    img = np.ascontiguousarray(img, np.uint8)
    with open(path, "wb") as f:
        if img.ndim == 2:
            f.write(b"P5\n%d %d\n255\n" % (img.shape[1], img.shape[0]))
            f.write(img.tobytes())
        else:
            f.write(b"P6\n%d %d\n255\n" % (img.shape[1], img.shape[0]))
            f.write(np.ascontiguousarray(img[:, :, ::-1]).tobytes())


class ImageSequence:
    def __init__(self, paths: Sequence[str]):
        self.paths = list(paths)

    def __len__(self):
        return len(self.paths)

    def read(self, i: int) -> np.ndarray:
        if not 0 <= i < len(self.paths):
            raise FrameError(f"frame {i} outside [0, {len(self.paths)})")
        p = self.paths[i]
        if p.lower().endswith((".pgm", ".ppm", ".pnm")):
            return read_pnm(p)
        try:
            from PIL import Image
        except ImportError as e:  # pragma: no cover
            raise FrameError(f"{p}: no reader for this format (Pillow missing)") from e
        im = Image.open(p)
        a = np.asarray(im.convert("L" if im.mode in ("L", "I;16") else "RGB"))
        return a if a.ndim == 2 else np.ascontiguousarray(a[:, :, ::-1])


class RawVideo:
    def __init__(self, path: str, rows: int, cols: int, fmt: str = "bgr24"):
        if fmt not in ("bgr24", "gray8"):
            raise ValueError("fmt must be bgr24 or gray8")
        ch = 3 if fmt == "bgr24" else 1
        self.shape = (rows, cols, 3) if ch == 3 else (rows, cols)
        size = os.path.getsize(path)
        self.frame_bytes = rows * cols * ch
        self.n = size // self.frame_bytes
        self._mm = np.memmap(path, np.uint8, "r", shape=(self.n,) + self.shape) if self.n else None

    def __len__(self):
        return self.n

    def read(self, i: int) -> np.ndarray:
        if not 0 <= i < self.n:
            raise FrameError(f"frame {i} outside [0, {self.n})")
        return np.array(self._mm[i])


class Y4MVideo:
    _CHROMA = {"444": (1, 1), "422": (2, 1), "420": (2, 2), "411": (4, 1), "mono": None}
    _SUFFIX_420 = ("", "jpeg", "paldv", "mpeg2")

    def __init__(self, path: str):
        self.path = path
        with open(path, "rb") as f:
            head = f.readline()
            if not head.startswith(b"YUV4MPEG2"):
                raise FrameError(f"{path}: not a YUV4MPEG2 stream")
            params = head.decode("ascii").split()[1:]
            d = {p[0]: p[1:] for p in params}
            self.cols, self.rows = int(d["W"]), int(d["H"])
            cs = d.get("C", "420jpeg")
            key = "mono" if cs.startswith("mono") else cs[:3]
            suffix = cs[len(key):]
            if key not in self._CHROMA:
                raise FrameError(f"{path}: chroma {cs} unsupported")
            # 8-bit sample layouts only: 420jpeg/paldv/mpeg2 differ in chroma
            # siting, not size; C420p10, C444p12, Cmono16 ... hold 16-bit
            # samples and 444alpha a fourth plane
            if suffix not in (self._SUFFIX_420 if key == "420" else ("",)):
                raise FrameError(f"{path}: chroma {cs} unsupported (8-bit "
                                 f"{'/'.join(sorted(self._CHROMA))} only)")
            sub = self._CHROMA[key]
            self.full_range = "XCOLORRANGE=FULL" in params
            luma = self.rows * self.cols
            chroma = 0 if sub is None else 2 * (-(-self.cols // sub[0])) * (-(-self.rows // sub[1]))
            self.frame_bytes = luma + chroma
            self.offsets: List[int] = []
            pos = len(head)
            size = os.path.getsize(path)
            while pos < size:
                f.seek(pos)
                line = f.readline()
                if not line.startswith(b"FRAME"):
                    raise FrameError(f"{path}: bad frame header at byte {pos}")
                data = pos + len(line)
                if data + self.frame_bytes > size:
                    break  # truncated last frame
                self.offsets.append(data)
                pos = data + self.frame_bytes

    def __len__(self):
        return len(self.offsets)

    def read(self, i: int) -> np.ndarray:
        """Gray frame: the luma plane (video range expanded to 0..255)."""
        if not 0 <= i < len(self.offsets):
            raise FrameError(f"frame {i} outside [0, {len(self.offsets)})")
        y = np.fromfile(self.path, np.uint8, count=self.rows * self.cols,
                        offset=self.offsets[i]).reshape(self.rows, self.cols)
        if self.full_range:
            return y
        g = (y.astype(np.int32) - 16) * 255 + 109          # round((Y-16)*255/219)
        return np.clip(np.floor_divide(g, 219), 0, 255).astype(np.uint8)


def write_y4m(path: str, frames: Iterable[np.ndarray], full_range: bool = True) -> None:
    """Gray frames as a 'Cmono' YUV4MPEG2 stream (test fixtures, examples)."""
    frames = list(frames)
    h, w = frames[0].shape
    with open(path, "wb") as f:
        f.write(b"YUV4MPEG2 W%d H%d F25:1 Ip A1:1 Cmono%s\n"
                % (w, h, b" XCOLORRANGE=FULL" if full_range else b""))
        for fr in frames:
            f.write(b"FRAME\n")
            f.write(np.ascontiguousarray(fr, np.uint8).tobytes())


def open_source(spec: str, rows: Optional[int] = None, cols: Optional[int] = None):
    """A path to .y4m, a raw .bgr/.rgb24/.gray file (needs rows, cols), or a
    directory / glob of image files (sorted)."""
    import glob
    low = spec.lower()
    if low.endswith(".y4m"):
        return Y4MVideo(spec)
    if low.endswith((".bgr", ".bgr24", ".gray", ".gray8")):
        if rows is None or cols is None:
            raise ValueError("raw video needs rows and cols")
        return RawVideo(spec, rows, cols, "gray8" if low.endswith((".gray", ".gray8"))
                        else "bgr24")
    paths = sorted(glob.glob(os.path.join(spec, "*")) if os.path.isdir(spec) else glob.glob(spec))
    if not paths:
        raise FrameError(f"{spec}: no frames")
    return ImageSequence(paths)


# ----------------------------------------------------------------- pairs
def capture_pair(src, prev: int, nxt: int) -> Tuple[np.ndarray, np.ndarray]:
    """main.cpp:53-59: seek to frame `prev`, read; seek to `nxt`, read; then
    the size check of :70-73."""
    a, b = src.read(prev), src.read(nxt)
    if a.shape[:2] != b.shape[:2]:
        raise FrameError("Image sizes are different")
    return a, b


def consecutive_pairs(n_frames: int, start: int = 0, count: Optional[int] = None,
                      gap: int = 1) -> List[Tuple[int, int]]:
    last = n_frames - gap
    idx = list(range(start, max(start, last)))
    if count is not None:
        idx = idx[:count]
    return [(j, j + gap) for j in idx]


def pair_windows(pairs: Sequence[Tuple[int, int]], size: int) -> List[List[int]]:
    """Indices of `pairs` cut into consecutive windows of at most `size`
    pairs (the unit solve_stream reads, uploads and solves at a time)."""
    size = max(1, int(size))
    return [list(range(k, min(len(pairs), k + size))) for k in range(0, len(pairs), size)]


def solve_stream(src, pairs: Sequence[Tuple[int, int]], window: int, iters: int,
                 alpha: float, rank: int = 0, world: int = 1, device=None, gather=True,
                 batch: int = 8, on_flow=None):
    """Frames -> pairs -> frame-parallel solve (main.cpp:53-59 over a stream
    of pairs).  The pairs go in windows of `batch` x world consecutive pairs:
    rank 0 reads only the frames a window needs (frames two pairs share --
    (j, j+1), (j+1, j+2) -- are read and converted once; the last frames
    carry over to the next window), uploads them as 8-bit BGR or gray,
    converts BGR to gray on the GPU (hsflow_bgr_to_gray_device), and the
    window runs through frame_parallel.run_stream_pipelined: each rank's
    share in batches of up to `batch` pairs (one batched flow_device call
    each, the batch rate of the resident bench rather than the single-pair
    one), scattered and gathered over torch.distributed when world > 1.
    Frames and device buffers of a window are released before the next, so
    device memory is bounded by the window, not by the video length.
    Returns rank 0's (u, v) per pair in order (device tensors; None on other
    ranks or when gather=False); with `on_flow(k, u, v)` each pair's flow is
    handed over as its window finishes and nothing is kept (memory bounded
    by one window of results too).  Bit-identical to one hsflow_flow call
    per pair (K1, K2 and K4 give the same bits for any batch)."""
    import torch
    import frame_parallel as fp
    import hsflow
    device = device or torch.device("cuda", torch.cuda.current_device())
    shape = None
    first = None
    if rank == 0 and pairs:
        first = src.read(pairs[0][0])
        shape = tuple(first.shape[:2])
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor(list(shape) if shape else [0, 0], dtype=torch.int64, device=device)
        dist.broadcast(t, 0)
        shape = (int(t[0]), int(t[1]))
    if not pairs:
        return [] if gather and rank == 0 else None
    rows, cols = shape
    ws = {"t": None, "n": 0}

    def solve_batch(I0, I1):
        n = I0.shape[0]
        if ws["n"] < n:  # one workspace for the largest batch, reused
            ws["t"] = hsflow.alloc_workspace(rows, cols, n, device)
            ws["n"] = n
        return hsflow.flow_device(I0, I1, window, iters, alpha, workspace=ws["t"])

    in_mb, out_mb = 2 * rows * cols / 1e6, 2 * rows * cols * 4 / 1e6

    def sizes(share):
        return fp.group_sizes(share, world, in_mb, out_mb, cap=batch)

    gray = {}

    def to_gray(i):
        nonlocal first
        if i not in gray:
            if first is not None and i == pairs[0][0]:  # read once, for the shape
                img, first = first, None
            else:
                img = src.read(i)
            x = torch.from_numpy(np.ascontiguousarray(img)).to(device)
            g = hsflow.bgr_to_gray_device(x) if x.dim() == 3 else x
            if tuple(g.shape) != shape:
                raise FrameError("Image sizes are different")  # main.cpp:70-73
            gray[i] = g
        return gray[i]

    out: List = []
    wins = pair_windows(pairs, batch * max(1, world))
    for w, idx in enumerate(wins):
        stream = None
        if rank == 0:
            stream = [(to_gray(pairs[k][0]), to_gray(pairs[k][1])) for k in idx]
        res = fp.run_stream_pipelined(stream, len(idx), shape, torch.uint8, solve_batch,
                                      device, rank, world, gather=gather, sizes=sizes)
        if rank == 0:
            # keep only the frames a later window reads
            later = ({f for k in wins[w + 1] for f in pairs[k]} if w + 1 < len(wins)
                     else set())
            for i in [i for i in gray if i not in later]:
                del gray[i]
            if gather and res is not None:
                for k, (u, v) in zip(idx, res):
                    if on_flow is not None:
                        on_flow(k, u, v)
                    else:
                        out.append((u, v))
    if rank != 0 or not gather:
        return None
    return None if on_flow is not None else out
