"""Summarise rocprofv3 output dirs (from scripts/gpu_prof.sh) into profiles/.

usage: python scripts/pmc_summary.py <prof_dir> <tag> [--workload 1080p --batch 8 --kb 6
        --fetch-scale S]
Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, verbatim) and
profiles/<tag>_pmc.json (per-dispatch medians for the dominant kernel), and
profiles/pmc_<workload>.json which bench.py reads for roofline.traffic,
hbm_frac and valu_frac.

HBM bytes = FETCH_SIZE*1024*fetch_scale + WRITE_SIZE*1024 (kB units).  The
fetch scale is the calibration of FETCH_SIZE for this kernel's access width
(profiles/r01_fetch_calibration.json: 2.0 for K2's 4-B and 8-B per-lane
buffer loads, as MI355X_MICROARCH.md §HBM states for 16-B loads).
Launch cycles = GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs; guide,
'DVFS give-back'); clock = launch cycles / the traced dispatch duration."""
import argparse, csv, collections, json, os, shutil, statistics

ap = argparse.ArgumentParser()
ap.add_argument("prof"); ap.add_argument("tag")
ap.add_argument("--workload", default="1080p"); ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--kb", type=int, default=6); ap.add_argument("--fetch-scale", type=float, default=2.0)
ap.add_argument("--kernel", default="hs_jacobi")
a = ap.parse_args()
root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
out = os.path.join(root, "profiles")
os.makedirs(out, exist_ok=True)
stats = os.path.join(a.prof, "trace", "run_kernel_stats.csv")
if os.path.exists(stats):
    shutil.copy(stats, os.path.join(out, f"{a.tag}_kernel_stats.csv"))
summary = {"kernel": a.kernel, "workload": a.workload, "batch": a.batch, "kb": a.kb,
           "counters": {}}
trace = os.path.join(a.prof, "trace", "run_kernel_trace.csv")
if os.path.exists(trace):
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
         for r in csv.DictReader(open(trace)) if a.kernel in r["Kernel_Name"]]
    summary["trace_avg_ns"] = statistics.mean(d)
    summary["trace_median_ns"] = statistics.median(d)
    summary["trace_dispatches"] = len(d)
for sub in sorted(os.listdir(a.prof)):
    f = os.path.join(a.prof, sub, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if a.kernel in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        summary["counters"][k] = statistics.median(v)
c = summary["counters"]
pmc = {"workload": a.workload, "batch": a.batch, "kb": a.kb,
       "source": f"profiles/{a.tag}_pmc.json"}
if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
    hbm = c["FETCH_SIZE"] * 1024 * a.fetch_scale + c["WRITE_SIZE"] * 1024
    summary["fetch_scale"] = a.fetch_scale
    summary["hbm_bytes_per_launch"] = pmc["hbm_bytes_per_launch"] = int(hbm)
if "GRBM_GUI_ACTIVE" in c:
    pmc["launch_cycles"] = summary["launch_cycles"] = c["GRBM_GUI_ACTIVE"] / 8
    if "trace_median_ns" in summary:
        pmc["clock_ghz"] = summary["clock_ghz"] = round(
            pmc["launch_cycles"] / summary["trace_median_ns"], 3)
if "SQ_INSTS_VALU" in c:
    pmc["valu_insts_per_launch"] = summary["valu_insts_per_launch"] = c["SQ_INSTS_VALU"]
if "hbm_bytes_per_launch" in pmc:
    json.dump(pmc, open(os.path.join(out, f"pmc_{a.workload}.json"), "w"), indent=1)
json.dump(summary, open(os.path.join(out, f"{a.tag}_pmc.json"), "w"), indent=1)
print(json.dumps(summary, indent=1))
