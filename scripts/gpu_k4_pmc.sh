#!/bin/bash
# K2 vs K4 Jacobi passes under rocprofv3: kernel trace + separate PMC passes
# (one counter group per run, each under its own time limit).
# usage: bash scripts/gpu_k4_pmc.sh <tag> [extra k2k4_passes.py args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for k in 2 4; do
  d=$out/k$k
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d/trace -o run --output-format csv -- \
      python3 scripts/k2k4_passes.py --kernel $k "$@" > $d.trace.log 2>&1 || exit 1
  i=0
  for ctr in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE" \
             "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $ctr -d $d/pmc$i -o run --output-format csv -- \
        python3 scripts/k2k4_passes.py --kernel $k "$@" > $d.pmc$i.log 2>&1 || exit 1
  done
done
echo done
