#!/bin/bash
# Counter passes for every roofline leg the default bench reports (single-
# stream launches: scripts/k2k4_passes.py) and for the bench's TIMED steps
# (step_*: scripts/timed_step.py, graph replays on the side streams), plus
# the FETCH_SIZE / WRITE_SIZE calibration, then profiles/pmc_<round>.json.
# usage (on the GPU box): bash scripts/gpu_pmc.sh ROUND [leg ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
rnd=${1:?round tag, e.g. r04}; shift
out=gpurun_out/pmc_$rnd; mkdir -p $out/calib
# bench.pmc_key name -> script arguments (bench.py WORKLOADS)
declare -A LEG=(
  [1080p_w5_b8]="--rows 1080 --cols 1920 --batch 8 --window 5 --iters 300"
  [4k_w5_b2]="--rows 2160 --cols 3840 --batch 2 --window 5 --iters 500"
  [1080p_w3_b8]="--rows 1080 --cols 1920 --batch 8 --window 3 --iters 300"
  [8k_w5_b1]="--rows 4320 --cols 7680 --batch 1 --window 5 --iters 1000 --f16"
  [1080p_w5_b1]="--rows 1080 --cols 1920 --batch 1 --window 5 --iters 300"
  [4k_w5_b1]="--rows 2160 --cols 3840 --batch 1 --window 5 --iters 500"
)
legs=${*:-"1080p_w5_b8 4k_w5_b2 1080p_w3_b8 8k_w5_b1 1080p_w5_b1 4k_w5_b1 step_1080p_w5_b8 step_4k_w5_b2 step_1080p_w5_b1"}
PASSES=("FETCH_SIZE" "WRITE_SIZE"
        "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
        "TCC_HIT_sum TCC_MISS_sum")

hipcc --offload-arch=gfx950 -O3 -o $out/fetch_calib scripts/ubench/fetch_calib.hip || exit 1
i=0
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $ctr -d $out/calib/pmc$i -o run --output-format csv -- \
      $out/fetch_calib > $out/calib.pmc$i.log 2>&1 || exit 1
done
for leg in $legs; do
  d=$out/$leg; mkdir -p $d
  if [[ $leg == step_* ]]; then
    args=${LEG[${leg#step_}]}
    [ -z "$args" ] && { echo "unknown leg $leg"; exit 1; }
    args=$(echo "$args" | sed 's/ --f16//')
    timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $d/trace -o run --output-format csv -- \
        python3 scripts/timed_step.py --reps 10 $args > $d.trace.log 2>&1 || exit 1
    i=0
    for ctr in FETCH_SIZE WRITE_SIZE; do
      i=$((i+1))
      timeout -s KILL 150 rocprofv3 --pmc $ctr -d $d/pmc$i -o run --output-format csv -- \
          python3 scripts/timed_step.py --reps 3 --warm-s 0 $args > $d.pmc$i.log 2>&1 || exit 1
    done
  else
    args=${LEG[$leg]}
    [ -z "$args" ] && { echo "unknown leg $leg"; exit 1; }
    timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $d/trace -o run --output-format csv -- \
        python3 scripts/k2k4_passes.py --kernel 0 --reps 1 $args > $d.trace.log 2>&1 || exit 1
    i=0
    for ctr in "${PASSES[@]}"; do
      i=$((i+1))
      timeout -s KILL 120 rocprofv3 --pmc $ctr -d $d/pmc$i -o run --output-format csv -- \
          python3 scripts/k2k4_passes.py --kernel 0 --reps 1 $args > $d.pmc$i.log 2>&1 || exit 1
    done
  fi
  echo "leg $leg done"
done
python3 scripts/pmc_collect.py $out $rnd
