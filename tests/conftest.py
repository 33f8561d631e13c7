"""Shared fixtures.  GPU tests are marked `gpu`; everything else runs on CPU."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
PKG = os.path.join(ROOT, "cpp-optical-flow_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


def read_pgm(path):
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(maxsplit=4)
    assert parts[0] == b"P5"
    w, h, mx = int(parts[1]), int(parts[2]), int(parts[3])
    assert mx == 255
    px = np.frombuffer(parts[4], np.uint8, count=w * h)
    return px.reshape(h, w)


@pytest.fixture(scope="session")
def golden_meta():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def kitti():
    """tag -> (gray prev, gray next), u8, from the reference's own frames."""
    out = {}
    for tag in ("000050", "000040"):
        out[tag] = (read_pgm(os.path.join(GOLDEN, f"kitti_{tag}_10.pgm")),
                    read_pgm(os.path.join(GOLDEN, f"kitti_{tag}_11.pgm")))
    return out


@pytest.fixture(scope="session")
def crop_small():
    return dict(np.load(os.path.join(GOLDEN, "crop64x48.npz")))


@pytest.fixture(scope="session")
def crop256():
    return dict(np.load(os.path.join(GOLDEN, "crop256.npz")))


def kat_labels(tag):
    z = np.load(os.path.join(GOLDEN, f"kat_{tag}.npz"))
    return z["labels"], z["ambiguous"]


def norm_rel_err(got, ref):
    """max|got-ref| / max|ref| (SURVEY §8c tolerance form)."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = max(float(np.max(np.abs(ref))), 1e-30)
    return float(np.max(np.abs(got - ref))) / scale


@pytest.fixture(scope="session")
def hs():
    """The product package (cpp-optical-flow_amd/hsflow.py over libhsflow.so)."""
    import hsflow
    return hsflow
