#!/bin/bash
# Kernel-trace profiles + bench lines at the C3 (10M) and C4-shape (100M) sizes, one GPU.
#   TAG=r02k TESTS="tests/test_pruned.py" bash tools/perf_pair.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${TAG:-pair}"
O=gpurun_out/$TAG
mkdir -p "$O"
step() { local name=$1 t=$2; shift 2; echo "[$name] $(date +%T)"; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; }
if [ -n "${TESTS:-}" ]; then
  step tests 600 python3 -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread
  tail -n 2 "$O/tests.log"
fi
for P in 10000000 100000000; do
  step prof_$P 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$P" -o run -- python3 bench.py --points $P --steps 3 --warmup 1 --no-secondary --no-extras --no-cpu-baseline
  python3 tools/kstats.py "$O/prof_$P" 9
  step bench_$P 300 python3 bench.py --points $P --steps 10 --warmup 2 --no-secondary --no-extras --no-cpu-baseline
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/bench_$P.log') if l.startswith('{')][-1]
r=d['roofline']
print('$P value',d['value'],'ms/step',d['ms_per_step'],'score avg ms',r['avg_launch_ms'],'mbp',r['memory_bound_passes']['frac'],r['memory_bound_passes']['ms_per_step'])
"
done
echo "done $(date +%T)"
