"""Summarise rocprofv3 output dirs (from scripts/gpu_prof.sh) into profiles/.

usage: python scripts/pmc_summary.py <prof_dir> <tag> [--workload 1080p --batch 8 --kb 4
        --fetch-scale S]
Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, verbatim) and
profiles/<tag>_pmc.json (per-dispatch medians for the dominant kernel), and
profiles/pmc_<workload>.json which bench.py reads for roofline.traffic.

HBM bytes = FETCH_SIZE*1024*fetch_scale + WRITE_SIZE*1024 (kB units).  The
fetch scale is the calibration of FETCH_SIZE for this kernel's access width
(dword buffer loads), measured by scripts/calib_fetch.py (MI355X_MICROARCH.md
§HBM: FETCH_SIZE under-reports 16-B/lane streams by 2x; other widths must be
calibrated)."""
import argparse, csv, collections, json, os, shutil, statistics

ap = argparse.ArgumentParser()
ap.add_argument("prof"); ap.add_argument("tag")
ap.add_argument("--workload", default="1080p"); ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--kb", type=int, default=4); ap.add_argument("--fetch-scale", type=float, default=1.0)
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
if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
    hbm = c["FETCH_SIZE"] * 1024 * a.fetch_scale + c["WRITE_SIZE"] * 1024
    summary["fetch_scale"] = a.fetch_scale
    summary["hbm_bytes_per_launch"] = int(hbm)
    json.dump({"workload": a.workload, "batch": a.batch, "kb": a.kb,
               "hbm_bytes_per_launch": int(hbm), "source": f"profiles/{a.tag}_pmc.json"},
              open(os.path.join(out, f"pmc_{a.workload}.json"), "w"), indent=1)
json.dump(summary, open(os.path.join(out, f"{a.tag}_pmc.json"), "w"), indent=1)
print(json.dumps(summary, indent=1))
