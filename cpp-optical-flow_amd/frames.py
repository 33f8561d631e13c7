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


def solve_stream(src, pairs: Sequence[Tuple[int, int]], window: int, iters: int,
                 alpha: float, rank: int = 0, world: int = 1, device=None, gather=True):
    """Frames -> pairs -> frame-parallel solve.  Rank 0 reads the frames
    (host I/O), uploads them as 8-bit BGR or gray and converts BGR to gray
    on the GPU; pairs are scattered round-robin over the ranks
    (frame_parallel.run_stream), solved with hsflow.flow_device and (u, v)
    gathered back in stream order on rank 0."""
    import torch
    import frame_parallel as fp
    import hsflow
    device = device or torch.device("cuda", torch.cuda.current_device())
    shape = None
    stream = None
    if rank == 0:
        gray = {}

        def to_gray(i):
            if i not in gray:
                fr = torch.from_numpy(np.ascontiguousarray(src.read(i))).to(device)
                gray[i] = hsflow.bgr_to_gray_device(fr) if fr.dim() == 3 else fr
            return gray[i]
        stream = [(to_gray(a), to_gray(b)) for a, b in pairs]
        shape = tuple(stream[0][0].shape)
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor(list(shape) if shape else [0, 0], dtype=torch.int64, device=device)
        dist.broadcast(t, 0)
        shape = (int(t[0]), int(t[1]))

    def solve(I0, I1):
        u, v = hsflow.flow_device(I0, I1, window, iters, alpha)
        return u, v
    return fp.run_stream(stream, len(pairs), shape, torch.uint8, solve, device, rank, world,
                         gather=gather)
