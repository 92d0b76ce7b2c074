#!/bin/bash
# One GPU session on the gpurun box: each GPU step under its own time limit; stop at the first
# step that crashes, aborts or times out (exit status other than 0/1).  Logs -> gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-smoke pytest bench}"
run() {
  local name=$1 t=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s"
  tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
python3 dialog_amd/build.py > gpurun_out/build.log 2>&1 || { echo "build failed"; tail gpurun_out/build.log; exit 2; }
for s in $STEPS; do
  case $s in
    smoke)  run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest_gpu 900 python3 -m pytest tests -m gpu -x -q -rA ;;
    pytestfast) run pytest_gpu 600 python3 -m pytest tests -m "gpu and not slow" -x -q ;;
    bench)  run bench 600 python3 bench.py ;;
    benchtorch) run bench_torch 600 python3 bench.py --torch-dist --no-cpu-baseline --steps 2 ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --steps 3 ;;
    pmc)    run pmc 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 ;;
    pmcw)   run pmcw 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "session done"
