set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03c5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_normals.py tests/test_normal_plane.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 -c "
import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(json.dumps(d['secondary']))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras > $O/prof_bench.log 2>&1
echo "prof rc=$?"
