"""Python host binding of libhsflow.so (MI355X Horn-Schunck).

Mirrors the reference's operator interface, HornSchunckOF/hornSchunck.cpp:

    hs = hornSchunck(windowSize, maxIterations, alpha)      # :13-17
    gx, gy, gt = hs.getGradients(imagePrev, imageNext)       # :19-41
    u, v = hs.getFlow(imagePrev, imageNext)                  # :43-75

with numpy arrays standing in for cv::Mat: inputs are 2-D uint8 / float16 /
float32 / float64 (any row stride), outputs are float64 (CV_64FC1, what the reference
returns and plotFlow.cpp:72-75 reads).  Also exposes the stream-ordered
device entry points for torch tensors and the host utilities.

Everything here calls the HIP path in libhsflow.so; there is no CPU fallback.
If the library is missing or no gfx950 device is present, calls raise.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

try:  # load torch's HIP runtime first so libhsflow binds to the same one
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the host API
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
# HSFLOW_LIB: load another build of the library (same-box A/B timing only)
LIB_PATH = os.environ.get("HSFLOW_LIB") or os.path.join(_HERE, "libhsflow.so")

HSFLOW_OK = 0
HSFLOW_ERR_ARG = -1
HSFLOW_ERR_HIP = -2
HSFLOW_ERR_OOM = -3
HSFLOW_ERR_NODEV = -4
HSFLOW_ERR_SIZE = -5
U8, F32, F64, F16 = 0, 1, 2, 3
MAX_LEVELS = 8

# every symbol include/hsflow.h declares
EXPORTS = (
    "hsflow_version", "hsflow_status_string", "hsflow_create", "hsflow_destroy",
    "hsflow_last_error", "hsflow_stream", "hsflow_flow", "hsflow_gradients",
    "hsflow_workspace_bytes", "hsflow_flow_device", "hsflow_gradients_device",
    "hsflow_jacobi_device", "hsflow_set_iters_per_launch", "hsflow_iters_per_launch",
    "hsflow_bgr_to_gray", "hsflow_synth_pair", "hsflow_set_max_streams",
    "hsflow_pyramid_level_size", "hsflow_pyramid_workspace_bytes",
    "hsflow_flow_pyramid_device", "hsflow_flow_pyramid", "hsflow_bgr_to_gray_device",
    "hsflow_flow_bgr", "hsflow_pyramid_build_device", "hsflow_upflow_device",
    "hsflow_set_jacobi_kernel", "hsflow_build_flags", "hsflow_flow_multi",
    "hsflow_download_device", "hsflow_jacobi_kernel_name", "hsflow_set_strip_rows",
    "hsflow_max_streams", "hsflow_set_output_hugepages", "hsflow_strip_seg_rows",
    "hsflow_flow_multi_release",
)


class HsflowError(RuntimeError):
    """A non-zero hsflow status (the reference would throw cv::Exception)."""

    def __init__(self, status: int, msg: str):
        super().__init__(f"hsflow status {status}: {msg}")
        self.status = status


_lib = None
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE, "-j4"])
    return LIB_PATH


def lib():
    """Load libhsflow.so (fails loudly if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `make -C {_HERE}` "
                          "(or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    i = ctypes.c_int
    L.hsflow_version.restype = i
    L.hsflow_status_string.restype = ctypes.c_char_p
    L.hsflow_status_string.argtypes = [i]
    L.hsflow_create.argtypes = [ctypes.POINTER(_vp), i]
    L.hsflow_destroy.argtypes = [_vp]
    L.hsflow_destroy.restype = None
    L.hsflow_last_error.argtypes = [_vp]
    L.hsflow_last_error.restype = ctypes.c_char_p
    L.hsflow_stream.argtypes = [_vp]
    L.hsflow_stream.restype = _vp
    L.hsflow_build_flags.restype = i
    L.hsflow_flow.argtypes = [_vp, _vp, _vp, i, i, i, _sz, _sz, i, i, ctypes.c_double,
                              _vp, _vp, i, _sz]
    L.hsflow_gradients.argtypes = [_vp, _vp, _vp, i, i, i, _sz, _sz, _vp, _vp, _vp, i,
                                   _sz]
    L.hsflow_workspace_bytes.argtypes = [i, i, i]
    L.hsflow_workspace_bytes.restype = _sz
    L.hsflow_flow_device.argtypes = [_vp, _vp, i, i, i, i, i, i, ctypes.c_float,
                                     _vp, _vp, _vp, _sz, _vp]
    L.hsflow_gradients_device.argtypes = [_vp, _vp, i, i, i, i, _vp, _vp, _vp,
                                          _vp, _sz, _vp]
    L.hsflow_jacobi_device.argtypes = [i, i, i, i, i, ctypes.c_float, i, _vp, _vp,
                                       _vp, _sz, _vp]
    L.hsflow_set_iters_per_launch.argtypes = [i]
    L.hsflow_iters_per_launch.argtypes = [i, i, i, i]
    L.hsflow_set_max_streams.argtypes = [i]
    L.hsflow_strip_seg_rows.argtypes = [i, i, i, i]
    L.hsflow_strip_seg_rows.restype = i
    L.hsflow_set_output_hugepages.argtypes = [i]
    L.hsflow_set_output_hugepages.restype = i
    L.hsflow_max_streams.argtypes = []
    L.hsflow_set_jacobi_kernel.argtypes = [i]
    L.hsflow_set_strip_rows.argtypes = [i]
    L.hsflow_jacobi_kernel_name.argtypes = [i, i, i, i]
    L.hsflow_jacobi_kernel_name.restype = ctypes.c_char_p
    L.hsflow_pyramid_level_size.argtypes = [i, i, i, ctypes.POINTER(i), ctypes.POINTER(i)]
    L.hsflow_pyramid_workspace_bytes.argtypes = [i, i, i, i]
    L.hsflow_pyramid_workspace_bytes.restype = _sz
    L.hsflow_flow_pyramid_device.argtypes = [_vp, _vp, i, i, i, i, i, i, i,
                                             ctypes.c_float, _vp, _vp, _vp, _sz, _vp]
    L.hsflow_flow_pyramid.argtypes = [_vp, _vp, _vp, i, i, i, _sz, _sz, i, i, i,
                                      ctypes.c_double, _vp, _vp, i, _sz]
    L.hsflow_pyramid_build_device.argtypes = [_vp, _vp, i, i, i, i, i,
                                              ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                                              _vp, _sz, _vp]
    L.hsflow_upflow_device.argtypes = [_vp, _vp, i, i, _vp, _vp, i, i, i, _vp]
    L.hsflow_bgr_to_gray_device.argtypes = [_vp, i, i, i, _vp, _vp]
    L.hsflow_flow_bgr.argtypes = [_vp, _vp, _vp, i, i, _sz, _sz, i, i, ctypes.c_double,
                                  _vp, _vp, i, _sz]
    L.hsflow_bgr_to_gray.argtypes = [_vp, i, i, _sz, _vp, _sz]
    L.hsflow_synth_pair.argtypes = [ctypes.c_uint64, i, i, i, i, _vp, _vp, _vp, _vp]
    L.hsflow_download_device.argtypes = [_vp, _vp, _sz, _vp]
    L.hsflow_flow_multi.argtypes = [ctypes.POINTER(i), i, i, ctypes.POINTER(_vp),
                                    ctypes.POINTER(_vp), i, i, i, _sz, _sz, i, i,
                                    ctypes.c_double, ctypes.POINTER(_vp),
                                    ctypes.POINTER(_vp), i, _sz]
    L.hsflow_flow_multi_release.argtypes = []
    L.hsflow_flow_multi_release.restype = None
    _lib = L
    return L


def _check(rc: int, ctx=None):
    if rc != HSFLOW_OK:
        L = lib()
        msg = L.hsflow_last_error(ctx).decode(errors="replace")
        raise HsflowError(rc, msg or L.hsflow_status_string(rc).decode())


def _dtype_code(a: np.ndarray) -> int:
    if a.dtype == np.uint8:
        return U8
    if a.dtype == np.float32:
        return F32
    if a.dtype == np.float64:
        return F64
    if a.dtype == np.float16:
        return F16
    raise HsflowError(HSFLOW_ERR_ARG, f"unsupported image dtype {a.dtype}")


def _common_dtype(a, b):
    """Frames of different element types are both widened to float64, as
    hornSchunck.cpp:23-24 converts each with convertTo(CV_64FC1); each frame
    keeps its own row step."""
    if a.dtype != b.dtype:
        return a.astype(np.float64), b.astype(np.float64)
    return a, b


def _as_image(a) -> np.ndarray:
    a = np.asarray(a)
    if a.ndim != 2:
        raise HsflowError(HSFLOW_ERR_ARG, "images must be single-channel 2-D "
                          "(convert BGR with bgr_to_gray, as main.cpp:13-14 does)")
    if a.strides[1] != a.itemsize or a.strides[0] < a.shape[1] * a.itemsize:
        a = np.ascontiguousarray(a)
    return a


def _reusable(out, shape, dtype) -> bool:
    """(u, v) can take a solve's output in place: the create() rule."""
    return all(isinstance(x, np.ndarray) and x.shape == tuple(shape) and
               x.dtype == np.dtype(dtype) and x.flags.c_contiguous and x.flags.writeable
               for x in out) and out[0] is not out[1]


class Context:
    """Device + stream + cached device buffers (hsflow_ctx)."""

    def __init__(self, device: int = 0):
        L = lib()
        p = _vp()
        rc = L.hsflow_create(ctypes.byref(p), int(device))
        if rc != HSFLOW_OK:
            raise HsflowError(rc, L.hsflow_last_error(None).decode(errors="replace"))
        self._p = p
        self.device = device

    @property
    def handle(self):
        return self._p

    def close(self):
        if getattr(self, "_p", None):
            lib().hsflow_destroy(self._p)
            self._p = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def flow(self, I0, I1, window: int, iters: int, alpha: float, out_dtype=np.float64,
             out=None):
        """getFlow on host arrays.  `out` = (u, v): C-contiguous rows x cols
        arrays of out_dtype written in place (cv::Mat::create() keeps an
        existing CV_64FC1 buffer of the right size the same way); else new
        arrays."""
        a, b = _as_image(I0), _as_image(I1)
        if a.shape != b.shape:
            raise HsflowError(HSFLOW_ERR_SIZE, "Image sizes are different")
        a, b = _common_dtype(a, b)
        rows, cols = a.shape
        if out is not None and _reusable(out, (rows, cols), out_dtype):
            u, v = out
        else:
            u = np.empty((rows, cols), out_dtype)
            v = np.empty((rows, cols), out_dtype)
        code = F64 if u.dtype == np.float64 else F32
        rc = lib().hsflow_flow(self._p, a.ctypes.data, b.ctypes.data, _dtype_code(a),
                               rows, cols, a.strides[0], b.strides[0], int(window),
                               int(iters),
                               float(alpha), u.ctypes.data, v.ctypes.data, code,
                               u.strides[0])
        _check(rc, self._p)
        return u, v

    def flow_pyramid(self, I0, I1, levels: int, window: int, iters: int, alpha: float,
                     out_dtype=np.float64):
        """Config 5 coarse-to-fine warm start (`iters` per level), see
        hsflow_flow_pyramid in include/hsflow.h."""
        a, b = _as_image(I0), _as_image(I1)
        if a.shape != b.shape:
            raise HsflowError(HSFLOW_ERR_SIZE, "Image sizes are different")
        a, b = _common_dtype(a, b)
        rows, cols = a.shape
        u = np.empty((rows, cols), out_dtype)
        v = np.empty((rows, cols), out_dtype)
        code = F64 if u.dtype == np.float64 else F32
        rc = lib().hsflow_flow_pyramid(self._p, a.ctypes.data, b.ctypes.data,
                                       _dtype_code(a), rows, cols, a.strides[0],
                                       b.strides[0], int(levels), int(window), int(iters), float(alpha),
                                       u.ctypes.data, v.ctypes.data, code, u.strides[0])
        _check(rc, self._p)
        return u, v

    def flow_bgr(self, bgr0, bgr1, window: int, iters: int, alpha: float,
                 out_dtype=np.float64):
        """main.cpp:50-51 + :13-14 + :97-98: decoded 8-bit BGR frames are
        uploaded as BGR and converted to gray on the GPU, then solved."""
        a = np.asarray(bgr0)
        b = np.asarray(bgr1)
        for x in (a, b):
            if x.dtype != np.uint8 or x.ndim != 3 or x.shape[2] != 3:
                raise HsflowError(HSFLOW_ERR_ARG, "need H x W x 3 BGR uint8")
        if a.shape != b.shape:
            raise HsflowError(HSFLOW_ERR_SIZE, "Image sizes are different")
        if a.strides[1:] != (3, 1) or a.strides[0] < 3 * a.shape[1]:
            a = np.ascontiguousarray(a)
        if b.strides[1:] != (3, 1) or b.strides[0] < 3 * b.shape[1]:
            b = np.ascontiguousarray(b)
        rows, cols = a.shape[:2]
        u = np.empty((rows, cols), out_dtype)
        v = np.empty((rows, cols), out_dtype)
        code = F64 if u.dtype == np.float64 else F32
        rc = lib().hsflow_flow_bgr(self._p, a.ctypes.data, b.ctypes.data, rows, cols,
                                   a.strides[0], b.strides[0], int(window), int(iters), float(alpha),
                                   u.ctypes.data, v.ctypes.data, code, u.strides[0])
        _check(rc, self._p)
        return u, v

    def gradients(self, I0, I1, out_dtype=np.float64):
        a, b = _as_image(I0), _as_image(I1)
        if a.shape != b.shape:
            raise HsflowError(HSFLOW_ERR_SIZE, "Image sizes are different")
        a, b = _common_dtype(a, b)
        rows, cols = a.shape
        gx, gy, gt = (np.empty((rows, cols), out_dtype) for _ in range(3))
        code = F64 if gx.dtype == np.float64 else F32
        rc = lib().hsflow_gradients(self._p, a.ctypes.data, b.ctypes.data, _dtype_code(a),
                                    rows, cols, a.strides[0], b.strides[0], gx.ctypes.data,
                                    gy.ctypes.data, gt.ctypes.data, code, gx.strides[0])
        _check(rc, self._p)
        return gx, gy, gt


_default_ctx = None


def download_device(dst, src, stream=None):
    """Stream-ordered download of the CUDA tensor `src` into the pinned host
    tensor `dst` (same byte size) through the runtime's DMA engines
    (hsflow_download_device), so it overlaps Jacobi passes running on other
    streams; torch's own copy_ of pinned memory runs as a blit kernel that
    takes their workgroup slots."""
    if src.numel() * src.element_size() != dst.numel() * dst.element_size():
        raise HsflowError(HSFLOW_ERR_ARG, "download sizes differ")
    if not (src.is_contiguous() and dst.is_contiguous()):
        raise HsflowError(HSFLOW_ERR_ARG, "download tensors must be contiguous")
    # a pageable dst would silently serialise the 'overlapped' copy, and a
    # CUDA dst would get a device-to-host copy kind on a device pointer
    if not src.is_cuda or dst.is_cuda or not dst.is_pinned():
        raise HsflowError(HSFLOW_ERR_ARG,
                          "download_device: src must be a CUDA tensor, dst pinned host memory")
    with _on(src.device):
        _check(lib().hsflow_download_device(dst.data_ptr(), src.data_ptr(),
                                            src.numel() * src.element_size(),
                                            _stream_ptr(stream, src.device)))


def flow_multi(devices, pairs, window: int, iters: int, alpha: float,
               out_dtype=np.float64):
    """Frame-parallel getFlow of host pairs over several GPUs from one
    process (hsflow_flow_multi): pair j on devices[j % len(devices)], one
    host thread + context per listed device.  `pairs`: list of (I0, I1)
    arrays of one shape and dtype.  Returns [(u, v), ...] in pair order."""
    pairs = [(_as_image(a), _as_image(b)) for a, b in pairs]
    if not pairs:
        return []
    rows, cols = pairs[0][0].shape
    dt, st0, st1 = pairs[0][0].dtype, pairs[0][0].strides[0], pairs[0][1].strides[0]
    for a, b in pairs:
        if a.shape != (rows, cols) or b.shape != (rows, cols):
            raise HsflowError(HSFLOW_ERR_SIZE, "Image sizes are different")
        if a.dtype != dt or b.dtype != dt or a.strides[0] != st0 or b.strides[0] != st1:
            raise HsflowError(HSFLOW_ERR_ARG, "pairs must share dtype and row steps")
    out = [(np.empty((rows, cols), out_dtype), np.empty((rows, cols), out_dtype))
           for _ in pairs]
    n = len(pairs)
    P = _vp * n
    devs = (ctypes.c_int * len(devices))(*devices)
    rc = lib().hsflow_flow_multi(
        devs, len(devices), n, P(*[a.ctypes.data for a, _ in pairs]),
        P(*[b.ctypes.data for _, b in pairs]), _dtype_code(pairs[0][0]), rows, cols, st0,
        st1, int(window), int(iters), float(alpha), P(*[u.ctypes.data for u, _ in out]),
        P(*[v.ctypes.data for _, v in out]), F64 if out_dtype == np.float64 else F32,
        out[0][0].strides[0])
    _check(rc)
    return out


def flow_multi_release():
    """Destroy the per-device contexts flow_multi keeps (hsflow_flow_multi_release)."""
    lib().hsflow_flow_multi_release()


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


class hornSchunck:  # noqa: N801  (reference class name, hornSchunck.cpp:8)
    """Drop-in mirror of `class hornSchunck` (hornSchunck.cpp:8-76)."""

    def __init__(self, inpWindowSize: int, inpMaxIterations: int, inpAlpha: float,
                 context: Context | None = None):
        # hornSchunck.cpp:13-17 -- public fields, same names
        self.windowSize = int(inpWindowSize)
        self.maxIterations = int(inpMaxIterations)
        self.alpha = float(inpAlpha)
        self._ctx = context

    def _c(self):
        return self._ctx if self._ctx is not None else default_context()

    def getGradients(self, imagePrev, imageNext, gradX=None, gradY=None, gradT=None):
        """hornSchunck.cpp:19-41 -> (gradX, gradY, gradT) float64."""
        gx, gy, gt = self._c().gradients(imagePrev, imageNext)
        for dst, src in ((gradX, gx), (gradY, gy), (gradT, gt)):
            if dst is not None:
                dst[...] = src
        return gx, gy, gt

    def getFlow(self, imagePrev, imageNext, u=None, v=None):
        """hornSchunck.cpp:43-75 -> (u, v) float64 (CV_64FC1).  Given u, v
        float64 arrays of the frame size, the solve writes into them (as the
        cv::Mat adapter's create() does); other arrays receive a copy."""
        out = (u, v) if u is not None and v is not None else None
        uu, vv = self._c().flow(imagePrev, imageNext, self.windowSize,
                                self.maxIterations, self.alpha, out=out)
        if u is not None and u is not uu:
            u[...] = uu
        if v is not None and v is not vv:
            v[...] = vv
        return uu, vv


def compute(I0, I1, alpha: float, nIter: int, windowSize: int = 5, levels: int = 1):
    """compute(I0, I1, alpha, nIter) -> (u, v): the north-star convenience
    wrapper over hornSchunck(windowSize, nIter, alpha).getFlow; levels > 1
    runs the config-5 coarse-to-fine warm start (nIter per level)."""
    if levels > 1:
        return default_context().flow_pyramid(I0, I1, levels, windowSize, nIter, alpha)
    return hornSchunck(windowSize, nIter, alpha).getFlow(I0, I1)


# ------------------------------------------------------------ device (torch)
def _stream_ptr(stream, device=None):
    """hipStream_t of `stream`, or of the current stream of `device` (the
    tensors' device) when stream is None.  The library runs a call on the
    device its stream belongs to; the null stream (torch's default stream is
    0 on every device) means the CURRENT device, so every wrapper below makes
    the tensors' device current around its library call (_on)."""
    if stream is None:
        return torch.cuda.current_stream(device).cuda_stream if torch is not None else None
    return getattr(stream, "cuda_stream", stream)


def _on(device):
    """Context that makes `device` current for one library call (a null
    stream runs on the current device, include/hsflow.h)."""
    return torch.cuda.device(device)


def build_flags() -> int:
    return int(lib().hsflow_build_flags())


def is_probe_build() -> bool:
    """True for a non-product build (hsflow_build_flags() != 0)."""
    return build_flags() != 0


def strip_seg_rows(rows: int, cols: int, batch: int = 1, window: int = 5) -> int:
    """hsflow_strip_seg_rows: K4 segment height a solve of this shape uses
    (0 when its full-depth passes run another kernel)."""
    return int(lib().hsflow_strip_seg_rows(rows, cols, batch, window))


def set_output_hugepages(on: bool) -> bool:
    """hsflow_set_output_hugepages: MADV_HUGEPAGE advice on f64 host outputs
    (default on; the advice stays on the caller's allocation).  Returns the
    previous setting."""
    return bool(lib().hsflow_set_output_hugepages(1 if on else 0))


def workspace_bytes(rows: int, cols: int, batch: int = 1) -> int:
    return int(lib().hsflow_workspace_bytes(rows, cols, batch))


def alloc_workspace(rows: int, cols: int, batch: int = 1, device="cuda"):
    n = workspace_bytes(rows, cols, batch)
    return torch.empty(n, dtype=torch.uint8, device=device)


def _tensor_dtype(t) -> int:
    if t.dtype == torch.uint8:
        return U8
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.float16:
        return F16
    if t.dtype == torch.float64:
        return F64
    raise HsflowError(HSFLOW_ERR_ARG,
                      f"device input dtype {t.dtype} (want uint8/float16/float32/float64)")


def _check_dense(t, shape, name):
    if not t.is_cuda or not t.is_contiguous() or tuple(t.shape[-2:]) != tuple(shape):
        raise HsflowError(HSFLOW_ERR_ARG, f"{name}: need a contiguous CUDA tensor "
                          f"[..., {shape[0]}, {shape[1]}]")


def _check_plane(t, shape, batch, name):
    """u, v (and the warm-start planes) are written by the kernels through
    raw pointers: a float32, contiguous CUDA tensor holding at least
    batch x rows x cols elements, or HsflowError (not a GPU fault)."""
    if t is None or not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous() or \
            tuple(t.shape[-2:]) != tuple(shape) or t.numel() < batch * shape[0] * shape[1]:
        raise HsflowError(HSFLOW_ERR_ARG, f"{name}: need a contiguous float32 CUDA tensor of "
                          f"{batch} x {shape[0]} x {shape[1]}")


def flow_device(I0, I1, window: int, iters: int, alpha: float, u=None, v=None,
                workspace=None, stream=None):
    """Stream-ordered solve on torch CUDA tensors [B, H, W] (or [H, W]).
    Returns (u, v) float32 tensors.  No host synchronisation."""
    rows, cols = I0.shape[-2:]
    batch = int(np.prod(I0.shape[:-2])) if I0.dim() > 2 else 1
    _check_dense(I0, (rows, cols), "I0")
    _check_dense(I1, (rows, cols), "I1")
    if I1.dtype != I0.dtype or I1.shape != I0.shape:
        raise HsflowError(HSFLOW_ERR_SIZE, "I0/I1 differ in shape or dtype")
    if u is None:
        u = torch.empty(I0.shape, dtype=torch.float32, device=I0.device)
    if v is None:
        v = torch.empty(I0.shape, dtype=torch.float32, device=I0.device)
    _check_plane(u, (rows, cols), batch, "u")
    _check_plane(v, (rows, cols), batch, "v")
    if workspace is None:
        workspace = alloc_workspace(rows, cols, batch, I0.device)
    with _on(I0.device):
        rc = lib().hsflow_flow_device(I0.data_ptr(), I1.data_ptr(), _tensor_dtype(I0), rows,
                                      cols, batch, int(window), int(iters), float(alpha),
                                      u.data_ptr(), v.data_ptr(), workspace.data_ptr(),
                                      workspace.numel(), _stream_ptr(stream, I0.device))
    _check(rc)
    return u, v


def pyramid_level_size(rows: int, cols: int, level: int):
    r, c = ctypes.c_int(), ctypes.c_int()
    _check(lib().hsflow_pyramid_level_size(rows, cols, level, ctypes.byref(r),
                                           ctypes.byref(c)))
    return r.value, c.value


def pyramid_workspace_bytes(rows: int, cols: int, batch: int, levels: int) -> int:
    return int(lib().hsflow_pyramid_workspace_bytes(rows, cols, batch, levels))


def flow_pyramid_device(I0, I1, levels: int, window: int, iters: int, alpha: float,
                        u=None, v=None, workspace=None, stream=None):
    """Config 5: coarse-to-fine warm start on torch CUDA tensors [B, H, W]
    (uint8 / float16 / float32), `iters` Jacobi iterations per level."""
    rows, cols = I0.shape[-2:]
    batch = int(np.prod(I0.shape[:-2])) if I0.dim() > 2 else 1
    _check_dense(I0, (rows, cols), "I0")
    _check_dense(I1, (rows, cols), "I1")
    if I1.dtype != I0.dtype or I1.shape != I0.shape:
        raise HsflowError(HSFLOW_ERR_SIZE, "I0/I1 differ in shape or dtype")
    if u is None:
        u = torch.empty(I0.shape, dtype=torch.float32, device=I0.device)
    if v is None:
        v = torch.empty(I0.shape, dtype=torch.float32, device=I0.device)
    _check_plane(u, (rows, cols), batch, "u")
    _check_plane(v, (rows, cols), batch, "v")
    if workspace is None:
        n = pyramid_workspace_bytes(rows, cols, batch, levels)
        workspace = torch.empty(n, dtype=torch.uint8, device=I0.device)
    with _on(I0.device):
        rc = lib().hsflow_flow_pyramid_device(I0.data_ptr(), I1.data_ptr(), _tensor_dtype(I0),
                                              rows, cols, batch, int(levels), int(window),
                                              int(iters), float(alpha), u.data_ptr(),
                                              v.data_ptr(), workspace.data_ptr(),
                                              workspace.numel(), _stream_ptr(stream, I0.device))
    _check(rc)
    return u, v


def pyramid_build_device(I0, I1, levels: int, workspace=None, stream=None):
    """Levels 1..levels-1 of both frames (f32 tensors [B, h_l, w_l]), the
    same planes hsflow_flow_pyramid_device builds internally."""
    rows, cols = I0.shape[-2:]
    batch = int(np.prod(I0.shape[:-2])) if I0.dim() > 2 else 1
    _check_dense(I0, (rows, cols), "I0")
    _check_dense(I1, (rows, cols), "I1")
    lead = tuple(I0.shape[:-2])
    P0, P1 = [], []
    for l in range(1, levels):
        r, c = pyramid_level_size(rows, cols, l)
        P0.append(torch.empty(lead + (r, c), dtype=torch.float32, device=I0.device))
        P1.append(torch.empty(lead + (r, c), dtype=torch.float32, device=I0.device))
    if workspace is None:
        workspace = alloc_workspace(rows, cols, batch, I0.device)
    n = max(1, levels - 1)
    a0 = (_vp * n)(*[t.data_ptr() for t in P0]) if P0 else (_vp * 1)()
    a1 = (_vp * n)(*[t.data_ptr() for t in P1]) if P1 else (_vp * 1)()
    with _on(I0.device):
        _check(lib().hsflow_pyramid_build_device(I0.data_ptr(), I1.data_ptr(), _tensor_dtype(I0),
                                                 rows, cols, batch, int(levels), a0, a1,
                                                 workspace.data_ptr(), workspace.numel(),
                                                 _stream_ptr(stream, I0.device)))
    return P0, P1


def upflow_device(uc, vc, u, v, stream=None):
    """u = 2 uc(y/2, x/2), v likewise (the pyramid's warm start); u, v and
    uc, vc are dense [rows, cols] / [rc, cc] views (row slices allowed)."""
    rc, cc = uc.shape[-2:]
    rows, cols = u.shape[-2:]
    for t, name, shape in ((uc, "uc", (rc, cc)), (vc, "vc", (rc, cc)), (u, "u", (rows, cols)),
                           (v, "v", (rows, cols))):
        _check_plane(t, shape, 1, name)
    with _on(u.device):
        _check(lib().hsflow_upflow_device(uc.data_ptr(), vc.data_ptr(), rc, cc, u.data_ptr(),
                                          v.data_ptr(), rows, cols, 1,
                                          _stream_ptr(stream, u.device)))


def gradients_device(I0, I1, workspace, gx=None, gy=None, gt=None, stream=None):
    rows, cols = I0.shape[-2:]
    batch = int(np.prod(I0.shape[:-2])) if I0.dim() > 2 else 1
    _check_dense(I0, (rows, cols), "I0")
    _check_dense(I1, (rows, cols), "I1")
    ptr = (lambda t: t.data_ptr() if t is not None else None)
    with _on(I0.device):
        rc = lib().hsflow_gradients_device(I0.data_ptr(), I1.data_ptr(), _tensor_dtype(I0),
                                           rows, cols, batch, ptr(gx), ptr(gy), ptr(gt),
                                           workspace.data_ptr(), workspace.numel(),
                                           _stream_ptr(stream, I0.device))
    _check(rc)


def jacobi_device(rows, cols, batch, window, iters, alpha, u, v, workspace,
                  warm_start=False, stream=None):
    _check_plane(u, (rows, cols), batch, "u")
    _check_plane(v, (rows, cols), batch, "v")
    with _on(u.device):
        rc = lib().hsflow_jacobi_device(int(rows), int(cols), int(batch), int(window),
                                        int(iters), float(alpha), int(bool(warm_start)),
                                        u.data_ptr(), v.data_ptr(), workspace.data_ptr(),
                                        workspace.numel(), _stream_ptr(stream, u.device))
    _check(rc)


def set_iters_per_launch(k: int):
    _check(lib().hsflow_set_iters_per_launch(int(k)))


def set_max_streams(n: int):
    """Side streams a batch is split over: 0 = automatic (2 for eager calls,
    none under stream capture), n >= 1 = up to n always."""
    _check(lib().hsflow_set_max_streams(int(n)))


def max_streams() -> int:
    """The current set_max_streams setting (0 = automatic)."""
    return int(lib().hsflow_max_streams())


class max_streams_as:
    """Context manager: set_max_streams(n) inside, the previous setting after."""

    def __init__(self, n: int):
        self.n = int(n)

    def __enter__(self):
        self.prev = max_streams()
        set_max_streams(self.n)
        return self

    def __exit__(self, *exc):
        set_max_streams(self.prev)
        return False


def set_jacobi_kernel(k: int):
    """Jacobi pass kernel: 0 = automatic (K4 streaming strips where built,
    K2 register tiles elsewhere), 2 = K2 everywhere, 4 = K4 where built;
    identical bits (include/hsflow.h)."""
    _check(lib().hsflow_set_jacobi_kernel(int(k)))


def set_strip_rows(seg_rows: int = 0):
    """K4 rows per segment (0 = automatic); identical bits for any choice."""
    _check(lib().hsflow_set_strip_rows(int(seg_rows)))


def jacobi_kernel_name(rows, cols, batch, window) -> str:
    """The kernel that runs this shape's full-depth Jacobi passes."""
    return lib().hsflow_jacobi_kernel_name(int(rows), int(cols), int(batch),
                                           int(window)).decode()


def iters_per_launch(rows, cols, batch, window) -> int:
    return int(lib().hsflow_iters_per_launch(rows, cols, batch, window))


# ------------------------------------------------------------------ host utils
def bgr_to_gray(bgr) -> np.ndarray:
    """main.cpp:13-14 cvtColor(BGR2GRAY), OpenCV 4.x 15-bit fixed point."""
    bgr = np.ascontiguousarray(bgr, np.uint8)
    if bgr.ndim != 3 or bgr.shape[2] != 3:
        raise HsflowError(HSFLOW_ERR_ARG, "need H x W x 3 BGR uint8")
    rows, cols = bgr.shape[:2]
    out = np.empty((rows, cols), np.uint8)
    _check(lib().hsflow_bgr_to_gray(bgr.ctypes.data, rows, cols, bgr.strides[0],
                                    out.ctypes.data, out.strides[0]))
    return out


def bgr_to_gray_device(bgr, gray=None, stream=None):
    """Device BGR->gray (same integer formula) on a uint8 CUDA tensor
    [..., H, W, 3] -> [..., H, W].  Stream-ordered."""
    if bgr.dtype != torch.uint8 or bgr.dim() < 3 or bgr.shape[-1] != 3 or \
            not bgr.is_cuda or not bgr.is_contiguous():
        raise HsflowError(HSFLOW_ERR_ARG, "need a contiguous uint8 CUDA tensor [..., H, W, 3]")
    rows, cols = bgr.shape[-3], bgr.shape[-2]
    batch = int(np.prod(bgr.shape[:-3])) if bgr.dim() > 3 else 1
    if gray is None:
        gray = torch.empty(bgr.shape[:-1], dtype=torch.uint8, device=bgr.device)
    if gray.dtype != torch.uint8 or not gray.is_cuda or not gray.is_contiguous() or \
            gray.numel() < batch * rows * cols or gray.device != bgr.device:
        raise HsflowError(HSFLOW_ERR_ARG, "gray: need a contiguous uint8 CUDA tensor of "
                          f"{batch} x {rows} x {cols} on {bgr.device}")
    with _on(bgr.device):
        _check(lib().hsflow_bgr_to_gray_device(bgr.data_ptr(), rows, cols, batch,
                                               gray.data_ptr(), _stream_ptr(stream, bgr.device)))
    return gray


def synth_pair(seed: int, rows: int, cols: int, qdy: int = -3, qdx: int = 6,
               dtype=np.float32):
    """Deterministic synthetic pair: motion (dy, dx) = (qdy, qdx)/4
    px, default (-0.75, +1.5).  Seed convention: 1000 + pair index."""
    I0 = np.empty((rows, cols), dtype)
    I1 = np.empty((rows, cols), dtype)
    if dtype == np.float32:
        args = (I0.ctypes.data, I1.ctypes.data, None, None)
    elif dtype == np.uint8:
        args = (None, None, I0.ctypes.data, I1.ctypes.data)
    else:
        raise HsflowError(HSFLOW_ERR_ARG, "synth dtype must be float32 or uint8")
    _check(lib().hsflow_synth_pair(int(seed), rows, cols, int(qdy), int(qdx), *args))
    return I0, I1
