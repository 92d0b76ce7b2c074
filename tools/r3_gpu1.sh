set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pcl_refit_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r03a/pcl_tests.log 2>&1
rc=$?; echo "pcl_tests rc=$rc"; tail -5 gpurun_out/r03a/pcl_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest tests/test_fullsize_golden.py -x -v -k "c3_extract or c2_segment" --timeout 300 --timeout-method thread > gpurun_out/r03a/full.log 2>&1
rc=$?; echo "full rc=$rc"; tail -5 gpurun_out/r03a/full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
DLG_TRACE=0 timeout -k 10 300 python -u bench.py --refit pcl --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-extras > gpurun_out/r03a/bench_pcl.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r03a/bench_pcl.log
