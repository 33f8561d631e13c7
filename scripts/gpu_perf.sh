set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc -> stop"; grep -E "^E |Error|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
for V in ${VARIANTS:-16 162 816 8162}; do
  HSFLOW_K2=$V timeout -k 10 300 python scripts/sweep.py --kbs ${KBS:-4,8} --workloads ${WLS:-1080p:8,4k:2} > gpurun_out/sweep_$V.log 2>&1 || exit $?
  echo "variant $V"; grep '^{' gpurun_out/sweep_$V.log
done
