#!/bin/bash
# A/B of the single-pass select tile size (DLG_OPT_SELECT_TILE) on the C3 and C4-shape benches;
# every GPU step under its own limit, the first failure ends the run.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-sel1ab}
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_pruned.py tests/test_gpu_parity.py tests/test_normal_plane.py tests/test_fast_refit_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1
for pts in ${POINTS:-10000000 100000000}; do
  for t in ${TILES:-16384 8192 4096}; do
    steps=10; [ "$pts" -gt 20000000 ] && steps=3
    timeout -k 10 300 python3 bench.py --points "$pts" --steps $steps --warmup 2 --no-extras --no-secondary \
      --no-cpu-baseline --select-tile "$t" > "$O/b_${pts}_$t.log" 2>&1
    python3 - "$O/b_${pts}_$t.log" "$pts" "$t" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
m = d['roofline']['memory_bound_passes']
print(sys.argv[2], sys.argv[3], 'value', d['value'], 'ms/step', d['ms_per_step'], 'select ms', m['ms_per_step'], 'frac', m['frac'])
PY
  done
done
