#!/bin/bash
# One measurement session on the GPU box (round 3): bench, kernel-trace stats, three PMC passes
# (FETCH_SIZE / WRITE_SIZE / SQ issue counters, one pass each as MI355X_MICROARCH.md prescribes),
# the derived profiles/score_traffic.json + profiles/score_issue.json, then the bench again so its
# JSON line carries them.  Every GPU step has its own time limit; the first failure ends the run.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${TAG:-r03}"
O=gpurun_out/$TAG
mkdir -p "$O"
B="python3 bench.py --steps 1 --warmup 0 --no-secondary --no-extras --no-cpu-baseline"
step() { local name=$1 t=$2; shift 2; echo "[$name] $(date +%T)"; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; }
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --steps 5 --warmup 2 --no-secondary --no-extras --no-cpu-baseline
step pmc_fetch 180 timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run -- $B
step pmc_write 180 timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run -- $B
step pmc_sq 180 timeout -s KILL 170 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/pmc_sq" -o run -- $B
F=$(find "$O/pmc_fetch" -name '*counter_collection.csv' -print -quit)
W=$(find "$O/pmc_write" -name '*counter_collection.csv' -print -quit)
S=$(find "$O/pmc_sq" -name '*counter_collection.csv' -print -quit)
python3 tools/traffic.py "$F" "$W" "$O/pmc_fetch.log" > "$O/traffic.log" 2>&1
python3 tools/pmc_issue.py "$S" > "$O/issue.log" 2>&1
cp profiles/score_traffic.json profiles/score_issue.json "$O/"
step bench 900 python3 bench.py --steps 10 --warmup 3 --no-secondary
echo "done $(date +%T)"
