# SQ counters (one --pmc pass) + kernel trace for Jacobi-kernel variants.
# usage: CFGS="HSFLOW_JACOBI=2 HSFLOW_JACOBI=3,HSFLOW_K3_WAVES=2" bash scripts/sq_probe.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp HSFLOW_STREAMS=1
WL=${WL:-1080p}
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --roofline-reps 1 --workload $WL"
i=0
for C in $CFGS; do
  i=$((i+1)); P=gpurun_out/sq$i; mkdir -p $P; echo "$C" > $P/cfg.txt
  env ${C//,/ } timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d $P/sq -o run --output-format csv -- python3 $B > $P/sq.log 2>&1 || exit $?
  env ${C//,/ } timeout -s KILL 120 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE -d $P/sq2 -o run --output-format csv -- python3 $B > $P/sq2.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, collections, glob, os, statistics
for d in sorted(glob.glob("gpurun_out/sq*/")):
    cfg = open(d + "cfg.txt").read().strip()
    agg = collections.defaultdict(list)
    for f in glob.glob(d + "*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "jacobi" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(cfg, {k: round(statistics.median(v)) for k, v in sorted(agg.items())})
PY
