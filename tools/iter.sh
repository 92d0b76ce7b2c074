#!/bin/bash
# One build-measure iteration on the GPU box: the lean/pick/parity GPU tests, a C3 bench line,
# a kernel trace of the same workload, and (POINTS100=1) the C4-shape bench.  Each GPU step has
# its own limit; the first failure ends the run.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-iter}
mkdir -p "$O"
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python3 -u -m pytest tests/test_pruned.py tests/test_gpu_parity.py tests/test_normal_plane.py tests/test_fast_refit_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1
  tail -1 "$O/tests.log"
fi
timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-cpu-baseline --no-extras > "$O/bench.log" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-extras > "$O/prof.log" 2>&1
if [ "${POINTS100:-0}" = 1 ]; then
  timeout -k 10 300 python3 bench.py --points 100000000 --steps 3 --warmup 2 --no-secondary --no-cpu-baseline --no-extras > "$O/bench100.log" 2>&1
fi
for f in "$O"/bench*.log; do
  python3 - "$f" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
m = d['roofline']['memory_bound_passes']
print(sys.argv[1], 'value', d['value'], 'ms/step', d['ms_per_step'], 'score', d['score_ms_per_step_max_rank'], 'select', m['ms_per_step'], 'frac', m['frac'])
PY
done
