set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03ad}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_pruned.py tests/test_fsum_gpu.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 -c "
import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], d.get('incl_index_build'), d.get('refit_fast'))"
