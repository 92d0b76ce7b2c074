set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_normals.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/knn_probe.py > $O/kt.log 2>&1 || exit 1
python3 -c "
import csv
r=list(csv.DictReader(open('$O/kt/run_kernel_trace.csv')))
r.sort(key=lambda x:int(x['Start_Timestamp']))
d=lambda x:(int(x['End_Timestamp'])-int(x['Start_Timestamp']))/1e6
print('knn', [round(d(x),2) for x in r if 'normals_knn' in x['Kernel_Name']])
print('cells_build', round(sum(d(x) for x in r if 'k_cells_build' in x['Kernel_Name']),2), 'cells_end', round(sum(d(x) for x in r if 'k_cells_end' in x['Kernel_Name']),2), 'all kernels', round(sum(d(x) for x in r),2), 'span', round((max(int(x['End_Timestamp']) for x in r)-min(int(x['Start_Timestamp']) for x in r))/1e6,2))
"
