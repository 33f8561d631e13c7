"""Does the kernel trace of a bench run account for its ms_per_step?

    rocprofv3 --kernel-trace --stats -d gpurun_out/bench_trace -o run \
        --output-format csv -- python3 bench.py --no-secondary --no-w3 --no-8k \
        --no-single --no-e2e --no-stream --no-cpu-baseline --no-bands --no-host-api > gpurun_out/bench_trace.json
    python scripts/trace_fit.py gpurun_out/bench_trace gpurun_out/bench_trace.json

The primary leg runs: one eager solve, a capture (no kernels execute), W
warm-up replays, K timed replays, then the roofline leg (K1 once, then
single-stream Jacobi passes).  Every solve starts with one gradient launch
(hs_gradients_kernel), so the trace splits into solves at those launches; the
K solves just before the roofline group are the timed steps.  For each, the
GPU span (first start to last end) and the busy time (union of kernel
intervals) are printed next to the bench's ms_per_step, the Jacobi kernels'
busy time per pass next to roofline.avg_launch_ms (the timed step's wall per
pass), and the roofline group's mean single-stream launch next to
roofline.isolated_launch.avg_launch_ms."""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    d, bench_json = sys.argv[1], sys.argv[2]
    line = [l for l in open(bench_json) if l.startswith("{")][-1]
    b = json.loads(line)
    steps = b["steps"]
    tr = []
    for f in glob.glob(os.path.join(d, "**", "run_kernel_trace.csv"), recursive=True):
        tr.extend(csv.DictReader(open(f)))
    ks = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"]),
                 x["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1]) for x in tr
                if "hs_" in x["Kernel_Name"])
    groups = []
    for k in ks:
        if k[2].startswith("hs_gradients_kernel") or not groups:
            groups.append([])
        groups[-1].append(k)
    # the roofline group: one gradient launch and > 2 solves' worth of passes
    counts = [len(g) for g in groups]
    roof_i = max(range(len(groups)), key=lambda i: counts[i])
    timed = groups[roof_i - steps:roof_i]

    def busy(g):
        t, end = 0, 0
        for s, e, _ in g:
            if e <= end:
                continue
            t += e - max(s, end)
            end = e
        return t

    spans = [max(e for _, e, _ in g) - g[0][0] for g in timed]
    res = {"ms_per_step_bench": b["ms_per_step"],
           "timed_solves_traced": len(timed),
           "kernels_per_solve": [len(g) for g in timed],
           "span_ms": [round(s / 1e6, 3) for s in spans],
           "busy_ms": [round(busy(g) / 1e6, 3) for g in timed],
           "span_ms_median": round(statistics.median(spans) / 1e6, 3)}
    res["span_over_bench_step"] = round(res["span_ms_median"] / b["ms_per_step"], 4)
    roof = b.get("roofline") or {}
    # the timed step's Jacobi kernels: busy time (union of the overlapping
    # half-batch launches) per pass against the bench's top-level
    # avg_launch_ms (= ms_per_step / passes)
    passes = roof.get("launches_per_solve")
    jbusy = [busy([k for k in g if k[2].startswith("hs_jacobi")]) for g in timed]
    res["timed_jacobi_busy_ms"] = [round(x / 1e6, 3) for x in jbusy]
    if passes:
        res["timed_jacobi_busy_ms_per_pass_median"] = round(
            statistics.median(jbusy) / 1e6 / passes, 5)
        res["roofline_avg_launch_ms_bench"] = roof.get("avg_launch_ms")
        res["trace_over_bench_per_pass"] = round(
            res["timed_jacobi_busy_ms_per_pass_median"] / roof["avg_launch_ms"], 4)
    jac = [e - s for s, e, n in groups[roof_i] if n.startswith("hs_jacobi")]
    res["isolated_group_launches"] = len(jac)
    res["isolated_mean_launch_ms_trace"] = round(statistics.mean(jac) / 1e6, 5)
    res["isolated_avg_launch_ms_bench"] = (roof.get("isolated_launch") or {}).get("avg_launch_ms")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
