"""Summarise rocprofv3 runs of the default bench command (scripts/gpu_prof_bench.sh)
into profiles/: the kernel trace of `python bench.py` exactly as the driver
runs it, and per-dispatch PMC counters from separate --pmc passes.

usage: python scripts/prof_bench.py <prof_dir> <tag>

K2 dispatches (hs_jacobi_wg_kernel) are grouped by grid: a 1080p launch has
323 tiles x 512 threads in X and its pairs in Y, a 4K launch 1258 tiles.  In
the default bench the timed legs split their batch over 2 side streams (Y = 4
at 1080p, 1 at 4K) and the roofline legs run single-stream (Y = 8, 2).
Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats, verbatim
  profiles/<tag>_profile.json        per-group durations, the timed solves'
                                     GPU wall time, per-dispatch counters
  profiles/pmc_<workload>.json       what bench.py reads (roofline.traffic,
                                     hbm_frac, valu_frac, step_hbm_frac)
HBM bytes = FETCH_SIZE*1024*2 + WRITE_SIZE*1024 (the x2: FETCH_SIZE
calibration for K2's 4- and 8-byte loads, profiles/r01_fetch_calibration.json);
launch cycles = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs).
"""
import collections
import csv
import json
import os
import shutil
import statistics
import sys

FETCH_SCALE = 2.0
TILES = {"1080p": 323 * 512, "4k": 1258 * 512}
LEGS = {("1080p", 4): "timed 2-stream half batch", ("1080p", 8): "roofline single stream",
        ("4k", 1): "timed 2-stream half batch", ("4k", 2): "roofline single stream",
        ("1080p", 32): "stream leg (64 pairs)"}


def key_of(r):
    """(workload, pairs) of a K2 dispatch: the trace has the grid per axis,
    the counter file only the total thread count."""
    if r.get("Grid_Size_X"):
        gx, gy = int(r["Grid_Size_X"]), int(r.get("Grid_Size_Y") or 1)
        for wl, x in TILES.items():
            if gx == x:
                return wl, gy
        return None
    g = int(r.get("Grid_Size") or 0)
    for wl, x in TILES.items():
        if g and g % x == 0 and (wl, g // x) in LEGS:
            return wl, g // x
    return None


def main():
    prof, tag = sys.argv[1], sys.argv[2]
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
    out = os.path.join(root, "profiles")
    stats = os.path.join(prof, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(out, f"{tag}_kernel_stats.csv"))
    summary = {"command": "python bench.py (default)", "groups": {}}
    rows = list(csv.DictReader(open(os.path.join(prof, "trace", "run_kernel_trace.csv"))))
    k2 = [r for r in rows if "hs_jacobi_wg_kernel" in r["Kernel_Name"]]
    k1 = [r for r in rows if "hs_gradients_kernel" in r["Kernel_Name"]]
    groups = collections.defaultdict(list)
    for r in k2:
        k = key_of(r)
        if k:
            groups[k].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for k, v in sorted(groups.items()):
        d = [e - s for s, e in v]
        summary["groups"][f"{k[0]} x{k[1]}"] = {
            "leg": LEGS.get(k, "?"), "dispatches": len(d),
            "avg_us": round(statistics.mean(d) / 1e3, 2),
            "median_us": round(statistics.median(d) / 1e3, 2)}
    # timed solves: the first time-cluster of each timed group, in chunks of
    # 2 x launches_per_solve dispatches (2 side streams)
    lps = {"1080p": 50, "4k": 84}
    k1s = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in k1)
    for wl, half in (("1080p", 4), ("4k", 1)):
        v = sorted(groups.get((wl, half), []))
        if not v:
            continue
        cl = [v[0]]
        for s, e in v[1:]:
            if s - cl[-1][1] > 20_000_000:  # 20 ms gap: next leg
                break
            cl.append((s, e))
        n = 2 * lps[wl]
        solves = [cl[i:i + n] for i in range(0, len(cl) - n + 1, n)]
        walls = []
        busy = []
        for sv in solves:
            s0, e0 = sv[0][0], max(e for _, e in sv)
            g = [x for x in k1s if s0 - 2_000_000 <= x[0] <= s0]
            if g:
                s0 = min(s0, g[-1][0])
            walls.append((e0 - s0) / 1e6)
            busy.append(sum(e - s for s, e in sv) / 1e6)
        summary[f"{wl}_timed_solves"] = {
            "solves": len(walls), "gpu_ms_per_solve_last5": round(statistics.mean(walls[-5:]), 3),
            "k2_dispatch_ms_sum_per_solve_last5": round(statistics.mean(busy[-5:]), 3),
            "note": "wall = first K1 start to last K2 end of a solve; the dispatch sum "
                    "exceeds it because the two streams' launches overlap"}
    # counters
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in sorted(os.listdir(prof)):
        f = os.path.join(prof, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            if "hs_jacobi_wg_kernel" not in r["Kernel_Name"]:
                continue
            k = key_of(r)
            if k:
                ctr[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    # per-dispatch rows carry one counter each; values are per dispatch
    for k, cs in ctr.items():
        g = summary["groups"].setdefault(f"{k[0]} x{k[1]}", {"leg": LEGS.get(k, "?")})
        med = {c: statistics.median(v) for c, v in cs.items()}
        g["counters_median"] = med
        if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
            g["hbm_bytes_per_dispatch"] = int(med["FETCH_SIZE"] * 1024 * FETCH_SCALE +
                                              med["WRITE_SIZE"] * 1024)
        if "GRBM_GUI_ACTIVE" in med:
            g["dispatch_cycles"] = med["GRBM_GUI_ACTIVE"] / 8
    for wl, batch, half in (("1080p", 8, 4), ("4k", 2, 1)):
        g = summary["groups"].get(f"{wl} x{batch}", {})
        gh = summary["groups"].get(f"{wl} x{half}", {})
        if "hbm_bytes_per_dispatch" not in g:
            continue
        pmc = {"workload": wl, "batch": batch, "kb": 6, "source": f"profiles/{tag}_profile.json",
               "hbm_bytes_per_launch": g["hbm_bytes_per_dispatch"]}
        if "dispatch_cycles" in g and g.get("median_us"):
            pmc["launch_cycles"] = g["dispatch_cycles"]
            pmc["clock_ghz"] = round(g["dispatch_cycles"] / (g["median_us"] * 1e3), 3)
        if "SQ_INSTS_VALU" in g.get("counters_median", {}):
            pmc["valu_insts_per_launch"] = g["counters_median"]["SQ_INSTS_VALU"]
        if "hbm_bytes_per_dispatch" in gh:
            # one pass of the timed 2-stream solve = two half-batch dispatches
            pmc["step_hbm_bytes_per_pass"] = 2 * gh["hbm_bytes_per_dispatch"]
        json.dump(pmc, open(os.path.join(out, f"pmc_{wl}.json"), "w"), indent=1)
    json.dump(summary, open(os.path.join(out, f"{tag}_profile.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
