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
    normals) run normals_gpu 600 python3 -m pytest tests/test_normals.py -m gpu -x -q -rA ;;
    post)   run post_gpu 600 python3 -m pytest tests/test_postprocess.py -m gpu -x -q -rA ;;
    pbench) run pbench 600 python3 tools/bench_post.py ;;
    pprof)  run pprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pprof -o run -- python3 tools/bench_post.py 10000000 2 ;;
    nbench) run nbench 600 python3 tools/bench_normals.py ;;
    c5)     run c5 600 python3 tools/bench_c5.py ;;
    c5prof) run c5prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof -o run -- python3 tools/bench_c5.py 10000000 2 ;;
    nprof)  run nprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nprof -o run -- python3 tools/bench_normals.py 10000000 2 ;;
    trace)  DLG_TRACE=1 run trace 300 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ;;
    benchtorch) run bench_torch 600 python3 bench.py --torch-dist --no-cpu-baseline --steps 2 ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --no-secondary --steps 3 ;;
    pmc)    run pmc 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o run -- python3 bench.py --no-cpu-baseline --no-secondary --steps 1 --warmup 0 ;;
    pstats) PRUNE_STATS=1 KERNELS="${KERNELS:-2,1}" run pstats 300 python3 tools/score_ab.py 10000000 4096 2 ;;
    ptest)  run ptest 600 python3 -u -m pytest tests/test_pruned.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread ;;
    ldspmc) KERNELS=2 run ldspmc 300 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/ldspmc -o run -- python3 tools/score_ab.py 10000000 4096 1 ;;
    ab)     run score_ab 600 python3 tools/score_ab.py ;;
    list)   run counters 120 rocprofv3 -L ;;
    sqpmc)  KERNELS="${KERNELS:-0,2}" run sqpmc1 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sqpmc1 -o run -- python3 tools/score_ab.py 10000000 4096 1 && \
            KERNELS="${KERNELS:-0,2}" run sqpmc2 600 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM GRBM_COUNT --output-format csv -d gpurun_out/sqpmc2 -o run -- python3 tools/score_ab.py 10000000 4096 1 ;;
    pmcw)   run pmcw 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw -o run -- python3 bench.py --no-cpu-baseline --no-secondary --steps 1 --warmup 0 ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "session done"
