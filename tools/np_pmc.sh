set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/sq -o run -- python3 tools/bench_c5.py 10000000 1 > $O/sq.log 2>&1 || exit 1
python3 -c "
import csv, collections
sq=list(csv.DictReader(open('$O/sq/run_counter_collection.csv')))
agg=collections.defaultdict(lambda: collections.defaultdict(float)); nm={}
for x in sq:
    if 'score_tiles_rl<1024, true' in x['Kernel_Name']:
        agg[x['Dispatch_Id']][x['Counter_Name']]+=float(x['Counter_Value'])
tot=collections.defaultdict(float)
for v in agg.values():
    for a,b in v.items(): tot[a]+=b
print(len(agg), {a:int(b/len(agg)) for a,b in tot.items()})
"
