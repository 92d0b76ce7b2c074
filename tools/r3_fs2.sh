set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fsum_gpu.py tests/test_pcl_refit_gpu.py -x -v -s --timeout 240 --timeout-method thread > $O/fsum_gpu.log 2>&1
rc=$?; echo "fsum/pcl rc=$rc"; tail -4 $O/fsum_gpu.log; grep "float sums" $O/fsum_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_fullsize_golden.py -x -v --timeout 300 --timeout-method thread -k "c2 or c3" > $O/full.log 2>&1
rc=$?; echo "full rc=$rc"; tail -3 $O/full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > $O/bench_pcl.json 2> $O/bench_pcl.err
rc=$?; echo "bench rc=$rc"; tail -c 300 $O/bench_pcl.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-extras > $O/prof_bench.log 2>&1
echo "prof rc=$?"
