#!/bin/bash
# K4 A/B on one box: stream split x segment direction x segment height,
# through the probe build (HSFLOW_K4_DOWN=1: every segment downwards).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=gpurun_out/${1:-k4ab}.log; : > $L
P=cpp-optical-flow_amd/libhsflow_probe.so
for st in 0 2; do
  for dn in 0 1; do
    HSFLOW_LIB=$P HSFLOW_K4_DOWN=$dn timeout -k 10 200 python -u scripts/k4_sweep.py \
      --cases ${CASES:-1080p8,4k2} --windows 5 --rows-list 0,84,96 --streams $st --tag down$dn \
      2>&1 | grep -v amdgpu.ids >> $L || exit 1
  done
done
cat $L
