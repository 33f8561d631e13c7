"""ctypes wrapper over the CPU float64 oracle (oracle/libhsoracle.so).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.  Every function
restates the reference HornSchunckOF path (see hs_oracle.h for file:line).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# HSORACLE_LIB: another build of the same sources (tests/test_sanitizers.py
# points it at the ASan/UBSan build, oracle/Makefile `asan`)
_LIB_PATH = os.environ.get("HSORACLE_LIB") or os.path.join(_HERE, "libhsoracle.so")
_lib = None

_dp = ctypes.POINTER(ctypes.c_double)
_u8p = ctypes.POINTER(ctypes.c_uint8)


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE, os.path.basename(_LIB_PATH)])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        L.hso_bgr_to_gray.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, _u8p]
        L.hso_gradients.argtypes = [_dp, _dp, ctypes.c_int, ctypes.c_int, _dp, _dp, _dp]
        L.hso_flow.argtypes = [_dp, _dp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.c_int, ctypes.c_double, _dp, _dp, ctypes.c_int]
        L.hso_jacobi.argtypes = [_dp, _dp, _dp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_double, _dp, _dp, ctypes.c_int]
        L.hso_pyrdown.argtypes = [_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp]
        L.hso_integer_pair.argtypes = [_dp, _dp, ctypes.c_size_t]
        L.hso_flow_pyramid.argtypes = [_dp, _dp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_double, _dp,
                                       _dp, ctypes.c_int]
        L.hso_plot_bresenham.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, _dp, _dp,
                                         ctypes.c_int, ctypes.c_float, ctypes.c_int]
        _lib = L
    return _lib


def _d(a):
    return a.ctypes.data_as(_dp)


def _f64(img):
    # hornSchunck.cpp:23-24  convertTo(CV_64FC1)
    return np.ascontiguousarray(np.asarray(img), dtype=np.float64)


def bgr_to_gray(bgr: np.ndarray) -> np.ndarray:
    """main.cpp:13-14 (cvtColor BGR2GRAY, OpenCV 4.x 15-bit fixed point)."""
    bgr = np.ascontiguousarray(bgr, dtype=np.uint8)
    rows, cols, _ = bgr.shape
    out = np.empty((rows, cols), np.uint8)
    lib().hso_bgr_to_gray(bgr.ctypes.data_as(_u8p), rows, cols, bgr.strides[0],
                          out.ctypes.data_as(_u8p))
    return out


def gradients(I0, I1):
    """hornSchunck.cpp:19-41 -> (gradX, gradY, gradT) float64."""
    a, b = _f64(I0), _f64(I1)
    rows, cols = a.shape
    gx, gy, gt = (np.empty_like(a) for _ in range(3))
    lib().hso_gradients(_d(a), _d(b), rows, cols, _d(gx), _d(gy), _d(gt))
    return gx, gy, gt


def flow(I0, I1, window: int, iters: int, alpha: float, nthreads: int = 1):
    """hornSchunck.cpp:43-75 -> (u, v) float64."""
    a, b = _f64(I0), _f64(I1)
    rows, cols = a.shape
    u, v = np.empty_like(a), np.empty_like(a)
    lib().hso_flow(_d(a), _d(b), rows, cols, int(window), int(iters), float(alpha),
                   _d(u), _d(v), int(nthreads))
    return u, v


def jacobi(gx, gy, gt, u0, v0, window: int, iters: int, alpha: float, nthreads: int = 1):
    """hornSchunck.cpp:56-74 continued from (u0, v0)."""
    gx, gy, gt = _f64(gx), _f64(gy), _f64(gt)
    u, v = _f64(u0).copy(), _f64(v0).copy()
    rows, cols = gx.shape
    lib().hso_jacobi(_d(gx), _d(gy), _d(gt), rows, cols, int(window), int(iters),
                     float(alpha), _d(u), _d(v), int(nthreads))
    return u, v


def integer_pair(I0, I1) -> bool:
    a, b = _f64(I0), _f64(I1)
    return bool(lib().hso_integer_pair(_d(a), _d(b), a.size))


def pyrdown(img, round_int: bool):
    """One pyramid level down (MultiResolution.cpp:9-97 kernel, see hs_oracle.h)."""
    a = _f64(img)
    rows, cols = a.shape
    out = np.empty(((rows + 1) // 2, (cols + 1) // 2), np.float64)
    lib().hso_pyrdown(_d(a), rows, cols, int(bool(round_int)), _d(out))
    return out


def flow_pyramid(I0, I1, levels: int, window: int, iters: int, alpha: float,
                 nthreads: int = 1):
    """Config 5: coarse-to-fine warm start, `iters` per level -> (u, v) f64."""
    a, b = _f64(I0), _f64(I1)
    rows, cols = a.shape
    u, v = np.empty_like(a), np.empty_like(a)
    lib().hso_flow_pyramid(_d(a), _d(b), rows, cols, int(levels), int(window),
                           int(iters), float(alpha), _d(u), _d(v), int(nthreads))
    return u, v


def plot_bresenham(bgr, u, v, delta=20, scale=20.0, outlier=5):
    """plotFlow.cpp:68-88 (headless): returns the plotted BGR copy."""
    img = np.ascontiguousarray(bgr, dtype=np.uint8).copy()
    rows, cols, _ = img.shape
    u, v = _f64(u), _f64(v)
    lib().hso_plot_bresenham(img.ctypes.data_as(_u8p), rows, cols, _d(u), _d(v),
                             int(delta), float(scale), int(outlier))
    return img
