set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/calib; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib/f -o run --output-format csv -- python3 scripts/calib_fetch.py > gpurun_out/calib/f.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/calib/r -o run --output-format csv -- python3 scripts/calib_fetch.py > gpurun_out/calib/r.log 2>&1 || exit $?
grep calib_ gpurun_out/calib/f/run_counter_collection.csv | cut -d, -f8,16-17
grep calib_ gpurun_out/calib/r/run_counter_collection.csv | cut -d, -f8,16-17
