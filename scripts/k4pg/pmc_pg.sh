set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
out=gpurun_out/pmc_pg; mkdir -p $out
args="--kernel 4 --rows 2160 --cols 3840 --batch 1 --window 5 --iters 500 --reps 1"
for seg in 1 2; do
  d=$out/seg$seg; mkdir -p $d
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $d/trace -o run --output-format csv -- python3 scripts/k2k4_passes.py $args --segments $seg > $d.trace.log 2>&1 || exit 1
  i=0
  for ctr in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_IFETCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d $d/pmc$i -o run --output-format csv -- python3 scripts/k2k4_passes.py $args --segments $seg > $d.pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -5 $d.pmc$i.log; exit 1; }
  done
done
python3 scripts/k4_pmc_summary.py $out > $out/summary.json; cat $out/summary.json
