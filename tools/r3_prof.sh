set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03p
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03p/prof -o run -- python3 bench.py --refit ${REFIT:-pcl} --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-extras > gpurun_out/r03p/bench.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -c 600 gpurun_out/r03p/bench.log
find gpurun_out/r03p -name "*kernel_stats.csv" | head
