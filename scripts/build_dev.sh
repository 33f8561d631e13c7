#!/bin/bash
# Development library: window 5 / KB 6 only, extra -D flags from the command
# line, linked as cpp-optical-flow_amd/libhsflow_dev_<tag>.so (same-box A/B
# with HSFLOW_LIB; never the product).  usage: build_dev.sh TAG [-DFLAG ...]
set -e
cd "$(dirname "$0")/../cpp-optical-flow_amd"
TAG=$1; shift
D=build_dev/$TAG; mkdir -p $D
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-slp-vectorize -DHSFLOW_DEV_W=5 -DHSFLOW_DEV_KB=6 $*"
pids=()
for s in hsflow_kernels.hip hsflow_pyramid.hip hsflow_input.hip hsflow_api.cpp hsflow_host.cpp; do
  /opt/rocm/bin/hipcc $F -c csrc/$s -o $D/${s%.*}.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done  # set -e: a failed compile stops here
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o libhsflow_dev_$TAG.so $D/*.o -Wl,-rpath,/opt/rocm/lib
echo built libhsflow_dev_$TAG.so
