set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03reg}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_normals.py tests/test_reference_data.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
cat > $O/t.py <<'PY'
import sys, time, json
sys.path.insert(0, ".")
import dialog_amd as D
from dialog_amd.synth import SEED_BASE, plane_cloud
p, lab, planes = plane_cloud(10_000_000, 20, seed=SEED_BASE + 5)
ctx = D.Context(0)
rn = D.estimate_normals(p, radius=0.1, ctx=ctx)
D.regulate_normals(p, rn, 0, True, 0.1, ctx=ctx)
t0 = time.perf_counter()
r = D.regulate_normals(p, rn, 0, True, 0.1, ctx=ctx)
print(json.dumps({"regulate_r0.1_ms": (time.perf_counter() - t0) * 1e3, "reached": int(r[2])}), flush=True)
PY
timeout -k 10 300 python -u $O/t.py > $O/t.json 2>&1
rc=$?; echo "t rc=$rc"; cat $O/t.json | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $O/t.py > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
