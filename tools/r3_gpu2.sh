set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu_tests rc=$rc"; tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --refit pcl --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > $O/bench_pcl.json 2> $O/bench_pcl.err
rc=$?; echo "bench pcl rc=$rc"; tail -c 400 $O/bench_pcl.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --refit fast --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-extras > $O/bench_fast.json 2> $O/bench_fast.err
rc=$?; echo "bench fast rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --refit pcl --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-extras > $O/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"
find $O/prof -name "*kernel_stats.csv"
