set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG}
mkdir -p $O
timeout -k 10 300 python -u tools/fs_walk_stats.py 4 $O/ws.json > $O/ws.txt 2>&1
rc=$?; echo "ws rc=$rc"; grep -A9 "^2 \|^3 " $O/ws.txt
