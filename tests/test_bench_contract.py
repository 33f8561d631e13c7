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
    # a physical fraction: the algorithmic bytes of one blocked pass
    assert 0 < r["frac"] <= 1.0
    assert r["kernel"] in ("hs_jacobi_strip_kernel", "hs_jacobi_wg_kernel")
    assert "workload" in d["config"]
    # the timed output was checked after NaN-filling it before the steps
    assert d["parity"]["outputs_nan_filled_before_timing"] is True


def test_bench_refuses_diagnostic_environment():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.refuse_diagnostics({"PATH": "/bin", "HSFLOW_BENCH_BACKEND": "gloo"}) == []
    assert bench.refuse_diagnostics({"HSFLOW_ABLATE": "1", "HSFLOW_STREAMS": "1"}) == \
        ["HSFLOW_ABLATE", "HSFLOW_STREAMS"]
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")], cwd=ROOT,
                         env=dict(os.environ, HSFLOW_K2_TL="0"), capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 2 and "HSFLOW_K2_TL" in out.stderr
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]


def test_parity_check_against_an_oracle_golden():
    """bench.parity_check: the oracle's own result passes, a 2e-4 relative
    perturbation of one sampled pixel (or a NaN anywhere) fails."""
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    import oracle
    from synth_ref import synth_pair
    I0, I1 = synth_pair(1000, 40, 64)
    u, v = oracle.flow(I0, I1, 5, 30, 1.0)
    e = {"step": 4, "sum_u": float(u.sum()), "sum_v": float(v.sum()),
         "max_u": float(np.abs(u).max()), "max_v": float(np.abs(v).max())}
    golden = ("t", e, u[::4, ::4].astype(np.float32), v[::4, ::4].astype(np.float32))
    ok = bench.parity_check(u.astype(np.float32), v.astype(np.float32), golden)
    assert ok["ok"] is True and ok["max_rel_err"] < 1e-6
    bad = u.astype(np.float32).copy()
    bad[8, 12] += 2e-4 * e["max_u"]
    assert bench.parity_check(bad, v, golden)["ok"] is False
    nan = u.astype(np.float32).copy()
    nan[1, 1] = np.nan
    assert bench.parity_check(nan, v, golden)["ok"] is False
    assert bench.parity_check(u, v, None)["ok"] is None


def test_bench_golden_fixture_covers_the_bench_workloads():
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    for wl, window in (("1080p", 5), ("4k", 5), ("1080p", 3), ("4k", 3)):
        w = bench.WORKLOADS[wl]
        g = bench.golden_entry(w["rows"], w["cols"], w["iters"], window, 1, 1.0)
        assert g is not None, (wl, window)
        name, e, us, vs = g
        step = e["step"]
        assert us.shape == vs.shape == (-(-w["rows"] // step), -(-w["cols"] // step))
        assert np.isfinite(us).all() and float(np.abs(us).max()) <= e["max_u"] * (1 + 1e-6)
        # SURVEY §8d sanity: mean u ~ dx / 8 (Sobel scaling) for dx = +1.5 px
        assert 0.05 < e["sum_u"] / (w["rows"] * w["cols"]) < 0.3


def test_gpus_flag_is_authoritative_world_selection():
    """--gpus N decides the rank count (bench.world_from_env): no launcher
    and N > 1 -> bench.py starts N ranks itself; a launcher whose
    WORLD_SIZE disagrees -> refuse; never a silent one-GPU line."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.world_from_env(1, {}) == ("run", 1)
    assert bench.world_from_env(2, {}) == ("launch", 2)
    assert bench.world_from_env(8, {}) == ("launch", 8)
    assert bench.world_from_env(2, {"WORLD_SIZE": "2"}) == ("run", 2)
    assert bench.world_from_env(8, {"WORLD_SIZE": "1"}) == ("refuse", 1)
    assert bench.world_from_env(1, {"WORLD_SIZE": "4"}) == ("refuse", 4)


def test_gpus_2_without_a_launcher_starts_two_ranks():
    """`python bench.py --gpus 2 --launch-check` (no WORLD_SIZE) launches two
    rank processes through torch.distributed.run on 127.0.0.1; rank 0 prints
    n_gpus 2 after a gloo all-reduce that sees both ranks (the plumbing the
    driver's 8-GPU run relies on; no GPU work)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--launch-check"], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks_seen"] == 2
    assert lines[0]["launcher"] == "torch.distributed.run"


def test_gpus_mismatch_with_launcher_refuses():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 2 and "WORLD_SIZE=1" in out.stderr
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]


def test_pmc_profile_used_only_for_the_kernel_source_it_was_collected_on(tmp_path, monkeypatch):
    """bench.pmc_for: a committed counter profile feeds roofline.traffic only
    when kernel, blocking depth and the kernels' source md5 all match."""
    import json
    import bench
    md5 = bench.kernel_source_md5()
    e = {"kernel": "hs_jacobi_strip_kernel", "kb": 6, "hbm_bytes_per_launch": 1,
         "kernel_source_md5": md5}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"1080p_w5_b8": e}))
    monkeypatch.setattr(bench, "PMC_JSON", str(p))
    assert bench.pmc_for("1080p", 5, 8, 6, "hs_jacobi_strip_kernel") == e
    assert bench.pmc_for("1080p", 5, 8, 8, "hs_jacobi_strip_kernel") is None
    assert bench.pmc_for("1080p", 5, 8, 6, "hs_jacobi_wg_kernel") is None
    p.write_text(json.dumps({"1080p_w5_b8": dict(e, kernel_source_md5="0" * 32)}))
    assert bench.pmc_for("1080p", 5, 8, 6, "hs_jacobi_strip_kernel") is None


def test_committed_pmc_profile_matches_the_kernel_sources():
    """profiles/pmc_r06.json (what the bench's roofline reads) was collected
    on the current Jacobi kernel sources, for the timed step of the headline
    and 4K legs as well as the single-stream launches; its timed-step bytes
    per pass are physical (the step's HBM traffic within 1.3x the
    algorithmic bytes of its passes)."""
    import bench
    d = json.load(open(bench.PMC_JSON))
    md5 = bench.kernel_source_md5()
    for leg in ("1080p_w5_b8", "4k_w5_b2", "step_1080p_w5_b8", "step_4k_w5_b2"):
        assert d[leg]["kernel_source_md5"] == md5, leg
    for leg, (rows, cols, batch, passes) in {"step_1080p_w5_b8": (1080, 1920, 8, 50),
                                             "step_4k_w5_b2": (2160, 3840, 2, 84)}.items():
        e = d[leg]
        assert e["passes_per_solve"] == passes and e["kb"] == 6
        alg = rows * cols * batch * bench.PASS_BYTES_PER_PX
        assert 1.0 <= e["hbm_bytes_per_step"] / passes / alg <= 1.3, leg
