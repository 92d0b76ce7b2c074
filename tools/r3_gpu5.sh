set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03o}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_fsum_gpu.py tests/test_pcl_refit_gpu.py "tests/test_fullsize_golden.py" -k "fsum or pcl or refit" -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-extras > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 900 $O/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-extras > $O/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"
find $O/prof -name "*kernel_stats.csv"
