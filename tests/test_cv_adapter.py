"""include/hornSchunck.hpp -- the cv::Mat drop-in with the reference's
exact signatures (hornSchunck.cpp:8-75) -- compiled against a cv::Mat test
double (tests/cpp/cvstub: OpenCV is absent from this image) and run as
main.cpp:97-98 does.  CPU: it compiles.  GPU: its u, v (CV_64FC1) equal the
Python host API's bit for bit, for u8, ROI and CV_16U frames, an ROI prev
with a contiguous next (independent row steps), frames of different depths,
and an output buffer shared with another header (written in place, as
OpenCV's MatExpr assignment does); edited public fields are honoured; errors
surface as cv::Exception."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "tests", "cpp", "adapter_main.cpp")


def _build(tmp_path):
    exe = str(tmp_path / "adapter_main")
    lib = os.path.join(ROOT, "cpp-optical-flow_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror",
                           "-I", os.path.join(ROOT, "tests", "cpp", "cvstub"),
                           "-I", os.path.join(ROOT, "include"), SRC, "-o", exe,
                           "-L", lib, "-lhsflow", "-Wl,-rpath," + lib])
    return exe


def test_adapter_compiles_against_the_cv_mat_surface(tmp_path):
    assert os.path.exists(_build(tmp_path))


@pytest.mark.gpu
def test_adapter_matches_host_api(tmp_path):
    import hsflow
    exe = _build(tmp_path)
    out = str(tmp_path / "r")
    res = subprocess.run([exe, out], capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, (res.returncode, res.stdout, res.stderr)
    rows, cols = 90, 130
    a, b = hsflow.synth_pair(1000, rows, cols, dtype=np.uint8)

    def load(tag):
        d = np.fromfile(f"{out}_{tag}.bin", np.float64)
        return d[:rows * cols].reshape(rows, cols), d[rows * cols:].reshape(rows, cols)
    ctx = hsflow.Context(0)
    ref = ctx.flow(a, b, 5, 100, 1.0)
    for tag in ("u8", "roi", "u16", "roi_mixed", "mixed_depth", "alias"):
        u, v = load(tag)
        assert np.array_equal(u, ref[0]) and np.array_equal(v, ref[1]), tag
    u, v = load("w3n7")
    r2 = ctx.flow(a, b, 3, 7, 1.0)
    assert np.array_equal(u, r2[0]) and np.array_equal(v, r2[1])
    gx, gy = load("grad_xy")
    g = ctx.gradients(a, b)
    assert np.array_equal(gx, g[0]) and np.array_equal(gy, g[1])
    ctx.close()
