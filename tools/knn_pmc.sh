set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/knn_probe.py > $O/kt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/sq -o run -- python3 tools/knn_probe.py > $O/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fe -o run -- python3 tools/knn_probe.py > $O/fe.log 2>&1 || exit 1
echo done
