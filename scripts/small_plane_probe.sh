# Jacobi-kernel variants on small batches (one pair) and on the 8K pyramid,
# whose coarsest level is a single 1080p plane.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
EXTRA="--batch 1" CFGS="HSFLOW_K2_TL=-1 HSFLOW_K2_TL=0 HSFLOW_JACOBI=3" WLS="1080p 4k" bash scripts/env_ab.sh || exit $?
CFGS="HSFLOW_K2_TL=-1 HSFLOW_K2_TL=0 HSFLOW_JACOBI=3" WLS="8k" bash scripts/env_ab.sh
