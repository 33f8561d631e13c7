#!/bin/bash
# A/B of lab builds (cpp-optical-flow_amd/lab/libhsflow_TAG.so), alternated,
# then a bitwise comparison of their u planes.  bash scripts/lab/geom_ab.sh A B
# (SHAPES=tag,tag,... limits the shapes)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/geom
for r in 1 2; do for t in "$@"; do
  timeout -k 5 240 python -u scripts/lab/geom_probe.py $t gpurun_out/geom $SHAPES || exit 1
done; done
python3 - "$@" <<'PY'
import sys, glob, numpy as np
a, b = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"gpurun_out/geom/{a}_*.npy")):
    g = f.replace(f"/{a}_", f"/{b}_")
    print(f.split("/")[-1], "bit-identical" if np.array_equal(np.load(f), np.load(g)) else "DIFFERENT")
PY
rm -f gpurun_out/geom/*.npy
