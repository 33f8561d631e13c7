"""bench.py keeps the driver's contract: one JSON line with the metric fields,
a `roofline` object and a `cpu_baseline` object (the float64 port of
hornSchunck.cpp on a bounded sample)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"}
ROOFLINE = {"bound", "achieved", "peak", "unit", "frac", "traffic"}
CPU = {"value", "unit", "cores", "kind", "sample"}


def test_cpu_baseline_leg_shape():
    sys.path.insert(0, ROOT)
    import bench
    cb = bench.cpu_baseline(48, 64, 5, 1.0, 2)
    assert CPU <= set(cb)
    assert cb["kind"] == "port" and cb["cores"] == 1 and cb["unit"] == "Mpix*iter/s"
    assert cb["value"] > 0


@pytest.mark.gpu
def test_bench_prints_one_contract_line():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1",
                          "--warmup", "1", "--iters", "24", "--roofline-reps", "1",
                          "--cpu-iters", "1"], capture_output=True, text=True, timeout=600,
                         cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert REQUIRED <= set(d)
    assert ROOFLINE <= set(d["roofline"]) and CPU <= set(d["cpu_baseline"])
    assert d["n_gpus"] == 1 and d["higher_is_better"] is True and d["value"] > 0
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert "workload" in d["config"]
