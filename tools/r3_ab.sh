set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_fsum_gpu.py tests/test_pcl_refit_gpu.py "tests/test_fullsize_golden.py" -k "fsum or pcl or refit or device" -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_walk.sh
