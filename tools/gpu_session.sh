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
    pstats) DLG_PRUNE_STATS=1 VARIANTS="${VARIANTS:-20,19}" run pstats 300 python3 tools/score_ab.py 10000000 4096 2 ;;
    abocc)  DLG_PRUNE_OCC=4 VARIANTS=20 run abocc4 300 python3 tools/score_ab.py 10000000 4096 5 && \
            DLG_PRUNE_OCC=8 VARIANTS=20 run abocc8 300 python3 tools/score_ab.py 10000000 4096 5 ;;
    ptest)  run ptest 600 python3 -u -m pytest tests/test_pruned.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread ;;
    abk)    DLG_PRUNE_STATS=1 DLG_PRUNE_KERNEL=1 VARIANTS=20,19 run abk1 300 python3 tools/score_ab.py 10000000 4096 5 && \
            DLG_PRUNE_STATS=1 DLG_PRUNE_KERNEL=2 VARIANTS=20,19 run abk2 300 python3 tools/score_ab.py 10000000 4096 5 ;;
    ldspmc) VARIANTS=20 run ldspmc 300 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/ldspmc -o run -- python3 tools/score_ab.py 10000000 4096 1 ;;
    expm)   for kk in 2; do for ee in 0 1 2 3; do
              DLG_PRUNE_KERNEL=$kk DLG_PRUNE_EXP=$ee SCORE_AB_NOCHECK=1 VARIANTS=20 run expm_k${kk}_e${ee} 120 python3 tools/score_ab.py 10000000 4096 5 || exit 3
            done; done ;;
    chunk)  for cc in 2 4 8; do DLG_PRUNE_CHUNK=$cc VARIANTS=20,19 run chunk_$cc 120 python3 tools/score_ab.py 10000000 4096 5 || exit 3; done ;;
    bpc)    for bb in 1 2 4; do DLG_PRUNE_BPC=$bb VARIANTS=20,19 run bpc_$bb 120 python3 tools/score_ab.py 10000000 4096 5 || exit 3; done ;;
    ab)     run score_ab 600 python3 tools/score_ab.py ;;
    list)   run counters 120 rocprofv3 -L ;;
    sqpmc)  VARIANTS="${VARIANTS:-0,2}" run sqpmc1 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sqpmc1 -o run -- python3 tools/score_ab.py 10000000 4096 1 && \
            VARIANTS="${VARIANTS:-0,2}" run sqpmc2 600 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM GRBM_COUNT --output-format csv -d gpurun_out/sqpmc2 -o run -- python3 tools/score_ab.py 10000000 4096 1 ;;
    mpmc)   VARIANTS="${VARIANTS:-5,12}" run mpmc1 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_SALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/mpmc1 -o run -- python3 tools/score_ab.py 10000000 4096 1 && \
            VARIANTS="${VARIANTS:-5,12}" run mpmc2 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES --output-format csv -d gpurun_out/mpmc2 -o run -- python3 tools/score_ab.py 10000000 4096 1 ;;
    pmcw)   run pmcw 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw -o run -- python3 bench.py --no-cpu-baseline --no-secondary --steps 1 --warmup 0 ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "session done"
