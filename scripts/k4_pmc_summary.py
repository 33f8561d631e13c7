"""Summarise scripts/gpu_k4_pmc.sh output: per kernel, the median per-dispatch
duration (trace) and counters of the Jacobi pass launches.
usage: python scripts/k4_pmc_summary.py gpurun_out/<tag> [--fetch-scale 2]"""
import csv, glob, json, os, statistics, sys

d = sys.argv[1]
scale = 2.0
res = {}
for kdir in sorted(glob.glob(os.path.join(d, "*"))):
    if not os.path.isdir(kdir):
        continue
    k = os.path.basename(kdir)
    r = {}
    tr = glob.glob(os.path.join(kdir, "trace", "**", "run_kernel_trace.csv"), recursive=True)
    if tr:
        ds = [int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in csv.DictReader(open(tr[0]))
              if "hs_jacobi" in x["Kernel_Name"]]
        names = {x["Kernel_Name"].split("(")[0] for x in csv.DictReader(open(tr[0])) if "hs_jacobi" in x["Kernel_Name"]}
        r["kernels"] = sorted(names)
        r["dispatches"] = len(ds)
        r["median_us"] = statistics.median(ds) / 1e3
    ctr = {}
    for f in glob.glob(os.path.join(kdir, "pmc*", "**", "run_counter_collection.csv"), recursive=True):
        agg = {}
        for x in csv.DictReader(open(f)):
            if "hs_jacobi" in x["Kernel_Name"]:
                agg.setdefault(x["Counter_Name"], []).append(float(x["Counter_Value"]))
        for n, v in agg.items():
            ctr[n] = statistics.median(v)
    r["counters"] = ctr
    if "FETCH_SIZE" in ctr and "WRITE_SIZE" in ctr:
        r["hbm_MB"] = (ctr["FETCH_SIZE"] * 1024 * scale + ctr["WRITE_SIZE"] * 1024) / 1e6
        if "median_us" in r:
            r["hbm_TBps"] = r["hbm_MB"] / r["median_us"]
    if "GRBM_GUI_ACTIVE" in ctr and "median_us" in r:
        r["clock_GHz"] = ctr["GRBM_GUI_ACTIVE"] / 8 / (r["median_us"] * 1e3)
        if "SQ_INSTS_VALU" in ctr:
            r["valu_frac_2cyc"] = ctr["SQ_INSTS_VALU"] * 2 / 1024 / (ctr["GRBM_GUI_ACTIVE"] / 8)
    if "SQ_WAVE_CYCLES" in ctr:
        w = ctr["SQ_WAVE_CYCLES"]
        r["wait_any"] = ctr.get("SQ_WAIT_ANY", 0) / w
        r["wait_inst_any"] = ctr.get("SQ_WAIT_INST_ANY", 0) / w
        r["active_inst_any"] = ctr.get("SQ_ACTIVE_INST_ANY", 0) / w
    for nm in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC",
               "SQ_INST_CYCLES_VMEM"):
        if nm in ctr and "SQ_WAVE_CYCLES" in ctr:
            r[nm.lower() + "_frac"] = ctr[nm] / ctr["SQ_WAVE_CYCLES"]
    if "TCC_HIT_sum" in ctr:
        r["l2_hit"] = ctr["TCC_HIT_sum"] / max(1, ctr["TCC_HIT_sum"] + ctr["TCC_MISS_sum"])
    res[k] = r
print(json.dumps(res, indent=1))
