# Parity of the in-tree build (blocking-depth invariance, oracle), then a
# same-box A/B of two library builds x slab settings.  abx/old.so and
# abx/new2.so are built ad hoc (make, then copy) and not kept in the tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "bit_invariant or blocking or f32_gradient or batch_equals or oracle" > gpurun_out/vsum_tests.log 2>&1 || { tail -30 gpurun_out/vsum_tests.log; exit 1; }
tail -2 gpurun_out/vsum_tests.log
LIBS="abx/old.so abx/new2.so" CFGS="HSFLOW_K2_TL=-1 HSFLOW_K2_TL=0" WLS="1080p 4k" REPS="1 2" bash scripts/lib_env_ab.sh
LIBS="abx/old.so abx/new2.so" CFGS="HSFLOW_K2_TL=-1" WLS="1080p 4k" EXTRA="--window 3" bash scripts/lib_env_ab.sh
