#!/bin/bash
# One GPU session on the box (gpurun), as a list of named steps run in order; every step has its
# own time limit and the first failure ends the session (no GPU step after a fault or timeout).
#
#   TAG=r04a bash tools/gpu.sh tests=tests/test_pruned.py ab bench prof
#
# steps:
#   tests=<pytest args, comma-separated>  GPU tests (-m gpu), thread-method timeouts
#   gputests                              the whole -m gpu suite
#   smoke                                 __graft_entry__.smoke()
#   ab[=n,D,rounds]                       tools/score_ab.py (pruned exact vs bf16 tile scorers)
#   bench[=extra args, comma-separated]   bench.py --steps 10 --warmup 3 (+ args)
#   benchfull                             bench.py as the driver runs it (defaults)
#   prof[=extra bench args]               rocprofv3 --kernel-trace --stats over a short bench
#   pmclds                                LDS counters (instructions, bank conflicts, LDS-busy and
#                                         LDS-issue-stall cycles) of the scoring launch, one pass
#   pmc                                   FETCH/WRITE/SQ-issue PMC passes of the scoring launch
#                                         -> traffic.py / pmc_issue.py summaries
#   c5                                    tools/bench_c5.py (normals, RegulateNormal, chain)
#   c5prof                                rocprofv3 --kernel-trace --stats over tools/c5_kernels.py
#   knnprof                               rocprofv3 --kernel-trace --stats over tools/knn_probe.py
#                                         (one k = 20 estimation: per-level dispatches)
#   c5pmc                                 SQ issue counters (one PMC pass) over tools/bench_c5.py
#   walk                                  tools/fs_walk_stats.py (PCL float-sum walk counters)
#   walkab=<a.so,b.so>                    walk counters under two library builds, alternated
#                                         (tools/with_lib.py; A/B of walk variants)
#   py=<script,args...>                   any python script (comma-separated argv)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${TAG:-run}"
O=gpurun_out/$TAG
mkdir -p "$O"
# a line a minute under gpurun_out/ while a long step (the full-size tests) runs silently
( while true; do date +%T >> "$O/heartbeat.log"; sleep 60; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
B1="python3 bench.py --steps 1 --warmup 0 --no-secondary --no-extras --no-cpu-baseline"

run() {  # run <name> <seconds> <cmd...>: output to $O/<name>.log, stop the session on failure
  local name=$1 t=$2; shift 2
  echo "[$name] $(date +%T) $*"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -n 3 "$O/$name.log"
  if [ $rc -ne 0 ]; then echo "session stopped at $name"; exit $rc; fi
}

for s in "$@"; do
  name=${s%%=*}; arg=""; [ "$name" != "$s" ] && arg=${s#*=}
  case $name in
    tests) run tests_$(echo "$arg" | tr -c 'a-zA-Z0-9_\n' '_' | cut -c1-40) 900 \
             python3 -u -m pytest ${arg//,/ } -m gpu -x -v --timeout 240 --timeout-method thread ;;
    gputests) run gputests 1100 python3 -u -m pytest tests -m gpu -x -v --durations=15 --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    ab) run ab_$(echo "$arg" | tr -c 'a-zA-Z0-9_\n' '_' | cut -c1-30) 300 env PRUNE_STATS=1 python3 -u tools/score_ab.py ${arg//,/ } ;;
    bench) run bench_$(echo "$arg" | tr -c 'a-zA-Z0-9_\n' '_' | cut -c1-40)_$(echo "$arg" | md5sum | cut -c1-6) 900 \
             python3 -u bench.py --steps 10 --warmup 3 ${arg//,/ } ;;
    benchfull) run benchfull 900 python3 -u bench.py ;;
    prof) run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
            python3 bench.py --steps 5 --warmup 2 --no-secondary --no-extras --no-cpu-baseline ${arg//,/ } ;;
    pmc)
      run pmc_fetch 180 timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run -- $B1
      run pmc_write 180 timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run -- $B1
      run pmc_sq 180 timeout -s KILL 170 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/pmc_sq" -o run -- $B1
      F=$(find "$O/pmc_fetch" -name '*counter_collection.csv' -print -quit)
      W=$(find "$O/pmc_write" -name '*counter_collection.csv' -print -quit)
      S=$(find "$O/pmc_sq" -name '*counter_collection.csv' -print -quit)
      python3 tools/traffic.py "$F" "$W" "$O/pmc_fetch.log" > "$O/traffic.log" 2>&1
      python3 tools/pmc_issue.py "$S" > "$O/issue.log" 2>&1
      cp profiles/score_traffic.json profiles/score_issue.json "$O/" ;;
    pmcab)  # PMC passes over one score_ab launch set: issue, LDS, SALU views of the tile scorers
      A="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_SALU"
      Bc="SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAVES"
      run pmcab_a 180 timeout -s KILL 170 env KERNELS=${arg:-2,3} rocprofv3 --pmc $A --output-format csv -d "$O/pmcab_a" -o run -- python3 tools/score_ab.py 10000000 4096 1
      run pmcab_b 180 timeout -s KILL 170 env KERNELS=${arg:-2,3} rocprofv3 --pmc $Bc --output-format csv -d "$O/pmcab_b" -o run -- python3 tools/score_ab.py 10000000 4096 1
      python3 tools/pmc_kern.py k_score_tiles $(find "$O/pmcab_a" "$O/pmcab_b" -name '*counter_collection.csv') > "$O/pmcab.json" 2>&1
      cat "$O/pmcab.json" ;;
    c5) run c5 600 python3 -u tools/bench_c5.py ${arg//,/ } ;;
    pmclds)  # LDS-side counters of the scoring launch (one pass: 8 SQ + 1 GRBM)
      run pmc_lds 180 timeout -s KILL 170 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d "$O/pmc_lds" -o run -- $B1
      L=$(find "$O/pmc_lds" -name '*counter_collection.csv' -print -quit)
      python3 tools/pmc_kern.py k_score_tiles_ex,k_prune_supers "$L" > "$O/pmc_lds_summary.log" 2>&1 ;;
    c5prof) run c5prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c5prof" -o run -- \
              python3 tools/c5_kernels.py ${arg//,/ } ;;
    c5xprof) run c5xprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c5xprof" -o run -- \
              python3 tools/bench_c5.py 10000000 1 ;;
    knnprof) run knnprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/knnprof" -o run -- \
              python3 tools/knn_probe.py ;;
    walk) run walk 300 python3 -u tools/fs_walk_stats.py ${arg//,/ } ;;
    c5pmc) run c5pmc 220 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d "$O/c5pmc" -o run -- python3 tools/bench_c5.py 10000000 1 ;;
    walkab)
      a=${arg%%,*}; b=${arg#*,}
      for v in "$a" "$b" "$a" "$b"; do
        run walkab_$(basename "$v" .so) 150 python3 -u tools/with_lib.py "$v" tools/fs_walk_stats.py 4
      done ;;
    py) run py_$(basename "${arg%%,*}" .py)_$(echo "$arg" | md5sum | cut -c1-6) 900 python3 -u ${arg//,/ } ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
echo "done $(date +%T)"
