"""CPU tests of the C-ABI library: it loads, exports every symbol declared in
include/hsflow.h, validates arguments, and its host utilities are exact.
No GPU compute here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import hsflow
from conftest import GOLDEN, ROOT
from synth_ref import synth_pair as np_synth


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "hsflow.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(hsflow_\w+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    L = hsflow.lib()
    syms = header_symbols()
    assert len(syms) >= 16
    for s in syms:
        assert hasattr(L, s), f"libhsflow.so lacks {s}"
    assert sorted(hsflow.EXPORTS) == syms


def test_version_and_status_strings():
    L = hsflow.lib()
    assert L.hsflow_version() == 20000
    assert L.hsflow_status_string(0) == b"ok"
    assert L.hsflow_status_string(-5) == b"image sizes differ"


def test_workspace_bytes():
    n = hsflow.workspace_bytes(1080, 1920, 2)
    assert n >= 1080 * 1920 * 2 * 24
    assert hsflow.workspace_bytes(0, 10, 1) == 0
    assert hsflow.workspace_bytes(10, 10, 0) == 0


def test_iters_per_launch_policy():
    # measured defaults: K4 streams w 5 at 6 and w 3 at 8
    # iterations per pass where its waves fill the chip; launches too small
    # for it run K2, at 6 (w 5) when a launch has rounds of workgroups and
    # 8 when one round does not fill the chip
    assert hsflow.iters_per_launch(1080, 1920, 8, 5) == 6
    assert hsflow.iters_per_launch(2160, 3840, 1, 5) == 6
    assert hsflow.jacobi_kernel_name(2160, 3840, 1, 5) == "hs_jacobi_strip_kernel"
    assert hsflow.iters_per_launch(1080, 1920, 1, 5) == 8
    assert hsflow.jacobi_kernel_name(1080, 1920, 1, 5) == "hs_jacobi_wg_kernel"
    assert hsflow.iters_per_launch(1080, 1920, 1, 3) == 8
    try:
        hsflow.set_jacobi_kernel(2)
        assert hsflow.iters_per_launch(1080, 1920, 8, 5) == 6
        assert hsflow.iters_per_launch(1080, 1920, 1, 5) == 8
        assert hsflow.iters_per_launch(375, 1242, 1, 5) == 8
    finally:
        hsflow.set_jacobi_kernel(0)
    assert hsflow.iters_per_launch(1080, 1920, 1, 12) == 1
    with pytest.raises(hsflow.HsflowError):
        hsflow.set_iters_per_launch(-1)
    hsflow.set_iters_per_launch(2)
    assert hsflow.iters_per_launch(1080, 1920, 1, 5) == 2
    hsflow.set_iters_per_launch(0)
    with pytest.raises(Exception):
        hsflow._check(hsflow.lib().hsflow_iters_per_launch(0, 1920, 1, 5))


def test_jacobi_kernel_selector():
    """0 = automatic (K4 strips where built), 2 = K2 tiles, 4 = K4 where
    built; others rejected.  The kernel name follows the choice (no GPU
    call: the name comes from the launcher's own selection logic)."""
    for bad in (-1, 1, 3, 5, 99):
        with pytest.raises(hsflow.HsflowError):
            hsflow.set_jacobi_kernel(bad)
    try:
        hsflow.set_jacobi_kernel(2)
        assert hsflow.jacobi_kernel_name(1080, 1920, 8, 5) == "hs_jacobi_wg_kernel"
        hsflow.set_jacobi_kernel(4)
        assert hsflow.jacobi_kernel_name(1080, 1920, 8, 5) == "hs_jacobi_strip_kernel"
        assert hsflow.jacobi_kernel_name(1080, 1920, 8, 3) == "hs_jacobi_strip_kernel"
        # K4 is built for window 3 at KB 8 and window 5 at KB 4, 5 and 6
        assert hsflow.jacobi_kernel_name(1080, 1920, 8, 7) == "hs_jacobi_wg_kernel"
        assert hsflow.jacobi_kernel_name(1080, 1920, 8, 2) == "hs_jacobi_kernel"
        assert hsflow.jacobi_kernel_name(1080, 1920, 8, 15) == "hs_jacobi_generic_kernel"
        for kb in (4, 5):
            hsflow.set_iters_per_launch(kb)
            assert hsflow.jacobi_kernel_name(1080, 1920, 8, 5) == "hs_jacobi_strip_kernel"
        hsflow.set_iters_per_launch(3)  # a depth K4 is not built for: K2
        assert hsflow.jacobi_kernel_name(1080, 1920, 8, 5) == "hs_jacobi_wg_kernel"
        hsflow.set_iters_per_launch(4)
        assert hsflow.jacobi_kernel_name(1080, 1920, 8, 3) == "hs_jacobi_wg_kernel"
    finally:
        hsflow.set_iters_per_launch(0)
        hsflow.set_jacobi_kernel(0)
    assert hsflow.jacobi_kernel_name(2160, 3840, 2, 5) == "hs_jacobi_strip_kernel"
    assert hsflow.jacobi_kernel_name(0, 10, 1, 5) == ""
    with pytest.raises(hsflow.HsflowError):
        hsflow.set_strip_rows(-1)
    hsflow.set_strip_rows(48)
    hsflow.set_strip_rows(0)


def test_device_entry_points_validate_before_touching_the_gpu():
    L = hsflow.lib()
    # bad sizes / null pointers are rejected without any HIP call
    assert L.hsflow_flow_device(None, None, 1, 0, 10, 1, 5, 10, 1.0, None, None,
                                None, 0, None) == hsflow.HSFLOW_ERR_ARG
    assert L.hsflow_jacobi_device(10, 10, 1, 0, 1, 1.0, 0, 1, 1, 1, 10 ** 6,
                                  None) == hsflow.HSFLOW_ERR_ARG
    assert L.hsflow_jacobi_device(10, 10, 1, 5, 1, 1.0, 0, 1, 1, 1, 16,
                                  None) == hsflow.HSFLOW_ERR_ARG  # workspace too small
    assert L.hsflow_gradients_device(1, 1, 7, 10, 10, 1, None, None, None, 1, 10 ** 6,
                                     None) == hsflow.HSFLOW_ERR_ARG  # unknown dtype


def test_flow_multi_validates_before_touching_the_gpu():
    """hsflow_flow_multi (one process, several GPUs): bad device lists and
    null pair buffers are rejected on the host; an empty batch is a no-op."""
    L = hsflow.lib()
    i = ctypes.c_int
    P = ctypes.c_void_p * 1
    devs = (i * 1)(0)
    one = P(None)
    assert L.hsflow_flow_multi(devs, 0, 1, one, one, 0, 4, 4, 4, 4, 5, 1, 1.0, one, one,
                               2, 32) == hsflow.HSFLOW_ERR_ARG           # no devices
    assert L.hsflow_flow_multi(None, 1, 1, one, one, 0, 4, 4, 4, 4, 5, 1, 1.0, one, one,
                               2, 32) == hsflow.HSFLOW_ERR_ARG
    assert L.hsflow_flow_multi(devs, 1, 1, one, one, 0, 4, 4, 4, 4, 5, 1, 1.0, one, one,
                               2, 32) == hsflow.HSFLOW_ERR_ARG           # null frames
    assert "pair 0" in L.hsflow_last_error(None).decode()
    assert L.hsflow_flow_multi(devs, 1, 0, None, None, 0, 4, 4, 4, 4, 5, 1, 1.0, None,
                               None, 2, 32) == hsflow.HSFLOW_OK          # empty batch
    assert L.hsflow_flow_multi(devs, 1, -1, None, None, 0, 4, 4, 4, 4, 5, 1, 1.0, None,
                               None, 2, 32) == hsflow.HSFLOW_ERR_ARG


def test_download_device_validates_on_the_host():
    """hsflow_download_device: zero bytes is a no-op, null buffers are
    rejected before any runtime call."""
    L = hsflow.lib()
    assert L.hsflow_download_device(None, None, 0, None) == hsflow.HSFLOW_OK
    assert L.hsflow_download_device(None, 1, 8, None) == hsflow.HSFLOW_ERR_ARG
    assert L.hsflow_download_device(1, None, 8, None) == hsflow.HSFLOW_ERR_ARG


def test_host_api_rejects_null_context():
    L = hsflow.lib()
    assert L.hsflow_flow(None, 1, 1, 0, 4, 4, 4, 4, 5, 1, 1.0, 1, 1, 2, 32) == hsflow.HSFLOW_ERR_ARG


def test_product_library_ignores_the_environment():
    """The product libhsflow.so is not the probe build: no HSFLOW_* variable
    can change what it computes or what a bench times."""
    assert not hsflow.is_probe_build()


def test_bgr_to_gray_matches_reference_conversion():
    z = np.load(os.path.join(GOLDEN, "bgr_crop.npz"))
    assert np.array_equal(hsflow.bgr_to_gray(z["bgr"]), z["gray"])


@pytest.mark.parametrize("rows,cols,qdy,qdx", [(37, 53, -3, 6), (16, 16, 0, 0),
                                               (64, 40, 5, -7), (1, 1, -3, 6)])
def test_synth_pair_matches_numpy_twin(rows, cols, qdy, qdx):
    a0, a1 = hsflow.synth_pair(1000, rows, cols, qdy, qdx)
    b0, b1 = np_synth(1000, rows, cols, qdy, qdx)
    assert np.array_equal(a0, b0) and np.array_equal(a1, b1)
    u0, u1 = hsflow.synth_pair(1000, rows, cols, qdy, qdx, dtype=np.uint8)
    assert np.array_equal(u0.astype(np.float32), a0)


def test_synth_pair_statistics():
    I0, I1 = hsflow.synth_pair(1000, 256, 256)
    assert I0.min() >= 0 and I0.max() <= 255
    assert 25 < I0.std() < 55 and abs(I0.mean() - 128) < 8
    # I1 is I0 moved by (+1.5 cols, -0.75 rows): I1[r, c] ~ I0[r+0.75, c-1.5]
    err = np.abs(I1[10:-10, 10:-10] - 0.5 * (I0[11:-9, 8:-12] + I0[11:-9, 9:-11]))
    assert err.mean() < 6
    c0, c1 = hsflow.synth_pair(1001, 64, 64)
    assert not np.array_equal(c0, I0[:64, :64])


def test_header_is_plain_c_and_links_from_c(tmp_path):
    """include/hsflow.h compiles as C99 with -Wall -Werror and libhsflow.so
    links from C; GPU-free entry points answer (no device touched)."""
    import shutil
    import subprocess
    from conftest import ROOT
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("no C compiler")
    lib_dir = os.path.join(ROOT, "cpp-optical-flow_amd")
    exe = str(tmp_path / "abi_c99")
    subprocess.check_call([gcc, "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic",
                           "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "c", "abi_c99.c"), "-o", exe,
                           "-L", lib_dir, "-lhsflow", "-Wl,-rpath," + lib_dir])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout + out.stderr
    bad, g0, g1 = (int(x) for x in out.stdout.split())
    # OpenCV 4.x 15-bit BGR2GRAY of (B,G,R) = (10,20,30) and (200,100,0)
    assert (g0, g1) == ((9798 * 30 + 19235 * 20 + 3735 * 10 + 16384) >> 15,
                        (9798 * 0 + 19235 * 100 + 3735 * 200 + 16384) >> 15)


def test_batch_and_plane_limits_are_rejected_on_the_host():
    assert hsflow.workspace_bytes(10, 10, 65535) > 0
    assert hsflow.workspace_bytes(10, 10, 65536) == 0          # gridDim limit
    assert hsflow.workspace_bytes(1 << 14, (1 << 15) - 1, 1) > 0   # < 2^29 px: accepted
    assert hsflow.workspace_bytes(1 << 14, 1 << 15, 1) == 0        # 2^29 px: offsets overflow
    assert hsflow.workspace_bytes(4 * 65535, 8, 1) > 0             # tallest plane
    assert hsflow.workspace_bytes(4 * 65535 + 1, 8, 1) == 0        # gridDim.y of K1


def test_integration_c_snippets_compile(tmp_path):
    """Every ```c block of INTEGRATION.md compiles against include/hsflow.h
    (gcc, C99, warnings as errors): a snippet with a stale argument list --
    e.g. one row step where the v2.0 ABI takes two -- fails here."""
    import re
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```c\n(.*?)```", text, re.S)
    assert blocks, "no C snippets found"
    # the names the snippets use, declared as a caller would have them
    pre = """#include <stddef.h>
#include <stdint.h>
#include "hsflow.h"
void snippet(void);
void snippet(void) {
    int rows = 375, cols = 1242, batch = 1;
    size_t prev_step = 1242, next_step = 1242, bgr_prev_step = 3726, bgr_next_step = 3726;
    const uint8_t *prev = 0, *next = 0, *bgr_prev = 0, *bgr_next = 0;
    double *u = 0, *v = 0;
    void *stream = 0, *workspace = 0;
    hsflow_ctx *ctx = 0;
    (void)ctx; (void)rows; (void)cols; (void)batch; (void)prev_step; (void)next_step;
    (void)bgr_prev_step; (void)bgr_next_step; (void)prev; (void)next; (void)bgr_prev;
    (void)bgr_next; (void)u; (void)v; (void)stream; (void)workspace;
"""
    for k, b in enumerate(blocks):
        src = tmp_path / f"snippet{k}.c"
        src.write_text(pre + "{\n" + b + "\n}\n}\n")
        out = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-Wno-unused-variable",
                              "-fsyntax-only", "-I", os.path.join(ROOT, "include"), str(src)],
                             capture_output=True, text=True)
        assert out.returncode == 0, f"INTEGRATION.md C snippet {k}:\n{b}\n{out.stderr}"


def test_kernel_choice_rules_for_partial_fills():
    """The round-5 kernel choice for launches that fill part of the chip
    (w = 5; scripts/kernel_choice_sweep.py measured each case on the GPU,
    profiles/r05_kernel_choice_sweep*.txt): a single pair takes K4 when
    60- or 48-row segments fill 0.35 of the wave slots, a batch when 48-row
    segments fill 0.6; everything else keeps the 84-row rule.  The choice
    is host logic (no GPU call; without a device the library assumes
    MI355X's 256 CUs)."""
    strip, tiles = "hs_jacobi_strip_kernel", "hs_jacobi_wg_kernel"
    cases = {
        (640, 7680, 1): strip,    # config 5's 8K level-0 band at N = 8 (K4 +8 %)
        (1176, 7680, 1): strip,   # ... at N = 4
        (1176, 3840, 1): strip,   # a 4K-level band at N = 2 (K4 +16 %)
        (1440, 2560, 1): strip,   # a 1440p pair (K4 +9 %)
        (464, 3840, 1): tiles,    # small bands stay on K2 (K2 fastest there)
        (732, 3840, 1): tiles,
        (1080, 1920, 1): tiles,   # the reference's single 1080p pair
        (1080, 1920, 2): tiles,
        (1080, 1920, 3): strip,   # K4 at 48 rows, +11 % over K2
        (1080, 1920, 8): strip,   # the headline batch
        (720, 1280, 4): tiles,
        (375, 1242, 8): tiles,
        (2160, 3840, 1): strip,
        (2160, 3840, 2): strip,
    }
    for (rows, cols, batch), name in cases.items():
        assert hsflow.jacobi_kernel_name(rows, cols, batch, 5) == name, (rows, cols, batch)


def test_k4_segment_heights_for_partial_fills():
    """K4 segment heights (w = 5): a single pair whose waves run alone on
    their SIMDs takes the cost model's height, now also below 48 rows
    (round 6, profiles/r06_kb_sweep.txt: a 1440p pair at 36 rows, 1000
    waves, 15 % faster than at 48); the 4K pair keeps 84 (962 waves), the
    batches 84, a 1080p pair runs K2 (0)."""
    cases = {(1440, 2560, 1): 36, (2160, 3840, 1): 84, (1080, 1920, 8): 84,
             (2160, 3840, 2): 84, (1080, 1920, 1): 0, (640, 7680, 1): 60}
    for (rows, cols, batch), n in cases.items():
        assert hsflow.strip_seg_rows(rows, cols, batch, 5) == n, (rows, cols, batch)
    hsflow.set_strip_rows(48)
    try:
        assert hsflow.strip_seg_rows(2160, 3840, 1, 5) == 48
    finally:
        hsflow.set_strip_rows(0)
