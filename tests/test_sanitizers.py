"""SURVEY.md §5, the sanitizer row, on the CPU: the float64 oracle (the
checker every parity test leans on) under AddressSanitizer + UBSan, and the
library's host copy pool (cpp-optical-flow_amd/csrc/hsflow_pool.h) under
ThreadSanitizer.  GPU sanitizers are not available on this pool; these are
the host-side parts."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


def _gcc_lib(name):
    out = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True)
    path = out.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


def _asan_env():
    asan, ubsan = _gcc_lib("libasan.so"), _gcc_lib("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("gcc sanitizer runtimes not installed")
    subprocess.check_call(["make", "-s", "-C", ORACLE, "asan"])
    env = dict(os.environ)
    env.update(LD_PRELOAD=f"{asan}:{ubsan}",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               HSORACLE_LIB=os.path.join(ORACLE, "libhsoracle_asan.so"))
    return env


def test_oracle_kat_and_golden_tests_under_asan_ubsan():
    """The oracle's own tests -- the reference-plot KAT, the numpy golden
    (u, v), gradients, reflect-101 on tiny images, the pyramid and cvtColor
    restatements -- with every oracle call running in the ASan/UBSan build
    (any finding aborts the child)."""
    env = _asan_env()
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        "-m", "not gpu", "tests/test_oracle_golden.py",
                        "tests/test_pyramid.py", "-k", "oracle or golden or kat or reflect "
                        "or gradients or bgr or flow or jacobi or config1"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "AddressSanitizer" not in tail and "runtime error" not in tail, tail
    assert " passed" in r.stdout


def test_asan_build_is_live():
    """The instrumented oracle really checks: a call told the frame is larger
    than its buffer aborts with an AddressSanitizer report."""
    env = _asan_env()
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import numpy as np, oracle\n"
            "L = oracle.lib(); assert 'asan' in oracle._LIB_PATH\n"
            "a = np.zeros((4, 4)); g = np.zeros((4, 4))\n"
            "L.hso_gradients(oracle._d(a), oracle._d(a), 64, 64, oracle._d(g), oracle._d(g),"
            " oracle._d(g))\n" % ORACLE)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0 and "AddressSanitizer" in r.stderr, r.stderr[-2000:]


def test_host_copy_pool_under_tsan(tmp_path):
    """Several host threads submit jobs to the copy pool at once (as
    hsflow_flow_multi's per-device workers do): no data race, every item of
    every job runs exactly once, and a pool's destructor joins its workers."""
    if subprocess.run(["g++", "--version"], capture_output=True).returncode != 0:
        pytest.skip("no g++")
    exe = str(tmp_path / "pool_tsan")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread",
                           "-I", os.path.join(ROOT, "cpp-optical-flow_amd", "csrc"),
                           os.path.join(ROOT, "tests", "cpp", "pool_tsan.cpp"), "-o", exe])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe, "6", "400"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, r.stderr[-3000:]
    assert "0 wrong items" in r.stdout


def test_f64_widening_under_tsan(tmp_path):
    """The host half of an f64 download (hsflow_widen.h): the page pre-touch
    (one zero byte per page of the output rows) and the widening of the
    same rows never overlap (they once ran as one pool job whose
    items finish out of order), no data race under ThreadSanitizer, and
    every widened value survives."""
    if subprocess.run(["g++", "--version"], capture_output=True).returncode != 0:
        pytest.skip("no g++")
    exe = str(tmp_path / "widen_tsan")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread",
                           "-DHSFLOW_PLAIN_WIDEN",
                           "-I", os.path.join(ROOT, "cpp-optical-flow_amd", "csrc"),
                           os.path.join(ROOT, "tests", "cpp", "widen_tsan.cpp"), "-o", exe])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe, "30"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, r.stderr[-3000:]
    assert "0 wrong values" in r.stdout
