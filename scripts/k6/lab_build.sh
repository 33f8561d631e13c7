#!/bin/bash
# K6 development variants: libhsflow built with the resident TU compiled
# under development macros (timing probes only; wrong results by design for
# the NOWAIT/NORELOAD variants).  Usage: bash k6lab/build.sh NAME "-DMACRO ..."
set -e
cd "$(dirname "$0")/.."
name=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-slp-vectorize -Wall $* \
    -c csrc/hsflow_resident.hip -o k6lab/res_$name.o
objs=$(ls build/*.o | grep -v hsflow_resident.o)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o k6lab/libhsflow_$name.so $objs k6lab/res_$name.o -Wl,-rpath,/opt/rocm/lib
