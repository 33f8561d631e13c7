"""Turn the rocprofv3 output of scripts/gpu_pmc.sh into the committed
profiles the bench reads.

    python scripts/pmc_collect.py gpurun_out/pmc_r04 r04

Inputs (one directory per bench roofline leg, named like bench.pmc_key):
  <leg>/trace/**/run_kernel_trace.csv     kernel trace of the leg's passes
  <leg>/pmc<i>/**/run_counter_collection.csv   one counter set per pass
  <leg>.trace.log                          "kernel <name> kb <k> ..." line
  calib/pmc<i>/**/run_counter_collection.csv   scripts/ubench/fetch_calib.hip

Timed-step legs (directories step_<leg>: scripts/timed_step.py, the bench's
graph-replayed solve with the batch split over the side streams) give
hbm_bytes_per_step = the bytes of every dispatch of the run / the solves
the run executed (one eager, the pre-warm replays, the timed replays: all
identical), and from the kernel trace the per-solve busy time of the Jacobi
kernel (union of its overlapping launches) next to the script's own
event-timed ms_per_step.

Outputs (ROUND = r04, ...):
  profiles/pmc_ROUND.json      per leg: kernel, kb, median launch duration,
                               HBM bytes per launch (FETCH_SIZE corrected by
                               the measured factor for 8-B-per-lane buffer
                               loads, WRITE_SIZE likewise), VALU instructions
                               and shader cycles per launch, clock, L2 hit rate
  profiles/pmc_ROUND_calib.json  FETCH_SIZE / WRITE_SIZE over the known bytes
                               of 4/8/16-B-per-lane streams of 1 GiB
  profiles/ROUND_<leg>_kernel_stats.csv   rocprofv3 --stats of each leg's trace

The counters of a leg are medians over its Jacobi launches of the kernel the
bench reports (the first launch of a solve reads no (u, v) and a tail launch
may use another kernel; the median is the steady launch)."""
import csv
import glob
import json
import os
import re
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CALIB_BYTES = 1 << 30


def rows_of(pattern):
    out = []
    for f in sorted(glob.glob(pattern, recursive=True)):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def short(name):
    return name.split("(")[0].split("<")[0].replace("void ", "").strip().split("::")[-1]


def calibration(d):
    """FETCH_SIZE (KiB) x 1024 / bytes per dispatch for each width, in the
    fetch_calib.hip launch order rd<4>, rd<8>, rd<16>, wr<4>, wr<8>, wr<16>."""
    res = {}
    for ctr, kern in (("FETCH_SIZE", "rd"), ("WRITE_SIZE", "wr")):
        vals = {}
        for x in rows_of(os.path.join(d, "calib", "pmc*", "**", "run_counter_collection.csv")):
            if x["Counter_Name"] != ctr:
                continue
            m = re.search(r"\b%s<(\d+)>" % kern, x["Kernel_Name"])
            if m:
                vals.setdefault(int(m.group(1)), []).append(float(x["Counter_Value"]))
        for width, v in sorted(vals.items()):
            res[f"{ctr}_b{width * 8}_ratio"] = round(statistics.median(v) * 1024 / CALIB_BYTES, 4)
    return res


def leg_summary(ldir, calib, rnd):
    name = os.path.basename(ldir)
    log = open(ldir + ".trace.log").read() if os.path.exists(ldir + ".trace.log") else ""
    m = re.search(r"kernel (\S+) kb (\d+)", log)
    if not m:
        return None
    kernel, kb = m.group(1), int(m.group(2))
    tr = rows_of(os.path.join(ldir, "trace", "**", "run_kernel_trace.csv"))
    durs = [int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in tr
            if short(x["Kernel_Name"]) == kernel]
    ctr = {}
    for x in rows_of(os.path.join(ldir, "pmc*", "**", "run_counter_collection.csv")):
        if short(x["Kernel_Name"]) == kernel:
            ctr.setdefault(x["Counter_Name"], []).append(float(x["Counter_Value"]))
    ctr = {k: statistics.median(v) for k, v in ctr.items()}
    e = {"kernel": kernel, "kb": kb, "dispatches_traced": len(durs),
         "median_launch_us": round(statistics.median(durs) / 1e3, 2) if durs else None,
         "counters": {k: round(v, 1) for k, v in ctr.items()},
         "source": f"rocprofv3 separate --pmc passes of scripts/k2k4_passes.py "
                   f"(scripts/gpu_pmc.sh, leg {name}); FETCH_SIZE / WRITE_SIZE "
                   f"corrected by profiles/pmc_{rnd}_calib.json"}
    fr = calib.get("FETCH_SIZE_b64_ratio") or 0.5
    wr = calib.get("WRITE_SIZE_b64_ratio") or 1.0
    e["fetch_correction"] = round(1 / fr, 4)
    e["write_correction"] = round(1 / wr, 4)
    if "FETCH_SIZE" in ctr and "WRITE_SIZE" in ctr:
        e["hbm_bytes_per_launch"] = int(ctr["FETCH_SIZE"] * 1024 / fr + ctr["WRITE_SIZE"] * 1024 / wr)
        e["fetch_bytes_per_launch"] = int(ctr["FETCH_SIZE"] * 1024 / fr)
        e["write_bytes_per_launch"] = int(ctr["WRITE_SIZE"] * 1024 / wr)
    if "GRBM_GUI_ACTIVE" in ctr:
        # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles
        e["launch_cycles"] = ctr["GRBM_GUI_ACTIVE"] / 8
        if e["median_launch_us"]:
            e["clock_ghz"] = round(e["launch_cycles"] / (e["median_launch_us"] * 1e3), 3)
    if "SQ_INSTS_VALU" in ctr:
        e["valu_insts_per_launch"] = ctr["SQ_INSTS_VALU"]
    if "SQ_WAVES" in ctr:
        e["waves_per_launch"] = ctr["SQ_WAVES"]
    if "TCC_HIT_sum" in ctr and "TCC_MISS_sum" in ctr:
        e["l2_hit"] = round(ctr["TCC_HIT_sum"] / max(1.0, ctr["TCC_HIT_sum"] + ctr["TCC_MISS_sum"]), 4)
    stats = glob.glob(os.path.join(ldir, "trace", "**", "run_kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{rnd}_{name}_kernel_stats.csv"))
    return e


def busy_union(iv):
    """total length of the union of [start, end) intervals"""
    tot, cur_s, cur_e = 0, None, None
    for a, b in sorted(iv):
        if cur_e is None or a > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def step_summary(ldir, calib, rnd):
    """A timed-step leg (scripts/timed_step.py under rocprofv3)."""
    name = os.path.basename(ldir)
    log = open(ldir + ".trace.log").read() if os.path.exists(ldir + ".trace.log") else ""
    m = re.search(r"kernel (\S+) kb (\d+) passes (\d+) prewarm (\d+) reps (\d+) "
                  r"ms_per_step (\S+)", log)
    if not m:
        return None
    kernel, kb, passes = m.group(1), int(m.group(2)), int(m.group(3))
    reps, ms_step = int(m.group(5)), float(m.group(6))
    e = {"kernel": kernel, "kb": kb, "passes_per_solve": passes,
         "script_ms_per_step": ms_step,
         "source": f"rocprofv3 kernel trace + separate --pmc passes of scripts/timed_step.py "
                   f"(scripts/gpu_pmc.sh, leg {name}: the bench's hipGraph-replayed solve, "
                   f"batch split over the side streams); FETCH_SIZE / WRITE_SIZE corrected "
                   f"by profiles/pmc_{rnd}_calib.json"}
    # the trace run: timed replays are the last `reps` solves; a solve's
    # Jacobi dispatches are its passes on every side stream
    tr = rows_of(os.path.join(ldir, "trace", "**", "run_kernel_trace.csv"))
    jac = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in tr
                 if short(x["Kernel_Name"]) == kernel or "jacobi" in short(x["Kernel_Name"]))
    allk = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in tr)
    # every solve issues the same launches
    n_solves_trace = None
    m2 = re.search(r"prewarm (\d+)", log)
    if m2:
        n_solves_trace = 1 + int(m2.group(1)) + reps
    if n_solves_trace and jac:
        per_solve = len(jac) // n_solves_trace
        kper = len(allk) // n_solves_trace
        last_j = jac[-per_solve * reps:]
        last_a = allk[-kper * reps:]
        e["jacobi_launches_per_solve"] = per_solve
        e["trace_jacobi_busy_ms_per_step"] = round(busy_union(last_j) / reps / 1e6, 4)
        e["trace_all_kernels_busy_ms_per_step"] = round(busy_union(last_a) / reps / 1e6, 4)
        e["trace_span_ms_per_step"] = round((last_a[-1][1] - last_a[0][0]) / reps / 1e6, 4)
    # counter runs: bytes of every dispatch / solves executed
    fr = calib.get("FETCH_SIZE_b64_ratio") or 0.5
    wr = calib.get("WRITE_SIZE_b64_ratio") or 1.0
    tot = {}
    for i, ctr in ((1, "FETCH_SIZE"), (2, "WRITE_SIZE")):
        plog = ldir + f".pmc{i}.log"
        lg = open(plog).read() if os.path.exists(plog) else ""
        mm = re.search(r"prewarm (\d+) reps (\d+)", lg)
        if not mm:
            continue
        solves = 1 + int(mm.group(1)) + int(mm.group(2))
        vals = [float(x["Counter_Value"]) for x in
                rows_of(os.path.join(ldir, f"pmc{i}", "**", "run_counter_collection.csv"))
                if x["Counter_Name"] == ctr]
        tot[ctr] = sum(vals) / solves
    if "FETCH_SIZE" in tot and "WRITE_SIZE" in tot:
        e["fetch_bytes_per_step"] = int(tot["FETCH_SIZE"] * 1024 / fr)
        e["write_bytes_per_step"] = int(tot["WRITE_SIZE"] * 1024 / wr)
        e["hbm_bytes_per_step"] = e["fetch_bytes_per_step"] + e["write_bytes_per_step"]
    stats = glob.glob(os.path.join(ldir, "trace", "**", "run_kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{rnd}_{name}_kernel_stats.csv"))
    return e


def kernel_source_md5():
    sys.path.insert(0, ROOT)
    import bench
    return bench.kernel_source_md5()


def main():
    d, rnd = sys.argv[1], sys.argv[2]
    md5 = kernel_source_md5()
    calib = calibration(d)
    with open(os.path.join(ROOT, "profiles", f"pmc_{rnd}_calib.json"), "w") as f:
        json.dump({"bytes_per_dispatch": CALIB_BYTES, "source": "scripts/ubench/fetch_calib.hip",
                   **calib}, f, indent=1)
    out = {}
    for ldir in sorted(glob.glob(os.path.join(d, "*"))):
        base = os.path.basename(ldir)
        if os.path.isdir(ldir) and base != "calib":
            e = (step_summary(ldir, calib, rnd) if base.startswith("step_")
                 else leg_summary(ldir, calib, rnd))
            if e:
                e["kernel_source_md5"] = md5
                out[os.path.basename(ldir)] = e
    with open(os.path.join(ROOT, "profiles", f"pmc_{rnd}.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps({"calib": calib, "legs": {k: {kk: v[kk] for kk in
          ("kernel", "kb", "median_launch_us", "hbm_bytes_per_launch", "clock_ghz", "l2_hit",
           "hbm_bytes_per_step", "script_ms_per_step", "trace_jacobi_busy_ms_per_step")
          if kk in v} for k, v in out.items()}}, indent=1))


if __name__ == "__main__":
    main()
