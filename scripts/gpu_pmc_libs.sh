#!/bin/bash
# PMC passes over K4 (or K2) Jacobi launches for several library builds.
# usage: bash scripts/gpu_pmc_libs.sh <tag> "<name>=<lib path>[:kernel] ..." [k2k4_passes args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=$1; libs=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
for spec in $libs; do
  name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; k=4
  [ "$rest" != "$lib" ] && k=${rest##*:}
  d=$out/$name; mkdir -p $d
  HSFLOW_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d/trace -o run --output-format csv -- \
      python3 scripts/k2k4_passes.py --kernel $k "$@" > $d.trace.log 2>&1 || exit 1
  i=0
  for ctr in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES" \
             "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    HSFLOW_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc $ctr -d $d/pmc$i -o run --output-format csv -- \
        python3 scripts/k2k4_passes.py --kernel $k "$@" > $d.pmc$i.log 2>&1 || exit 1
  done
done
python3 scripts/k4_pmc_summary.py $out > $out/summary.json && cat $out/summary.json
