#!/bin/bash
# One GPU iteration on the box: the GPU tests named in $TESTS (default: the whole -m gpu suite),
# then a kernel-trace profile of a short C3 bench run and the bench line itself.  Every GPU step
# has its own time limit; the first failure ends the run.
#   TAG=r02b TESTS="tests/test_fast_refit_gpu.py" bash tools/gpu_iter.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${TAG:-iter}"
O=gpurun_out/$TAG
mkdir -p "$O"
step() { local name=$1 t=$2; shift 2; echo "[$name] $(date +%T)"; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; }
if [ "${TESTS:-all}" != "none" ]; then
  if [ "${TESTS:-all}" = "all" ]; then T="tests"; else T="$TESTS"; fi
  step tests 600 python3 -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread
  tail -n 2 "$O/tests.log"
fi
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --steps 5 --warmup 2 --no-secondary --no-extras --no-cpu-baseline ${BENCH_ARGS:-}
python3 tools/kstats.py "$O/prof" > "$O/kstats.txt" && cat "$O/kstats.txt"
step bench 600 python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline ${BENCH_ARGS:-}
python3 -c "
import json,sys
d=[json.loads(l) for l in open('$O/bench.log') if l.startswith('{')][-1]
r=d['roofline']
print('value',d['value'],'ms/step',d['ms_per_step'],'score avg ms',r['avg_launch_ms'],'mbp',r['memory_bound_passes']['frac'],r['memory_bound_passes']['ms_per_step'])
"
echo "done $(date +%T)"
