set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG}
mkdir -p $O
for v in a b a b; do
  timeout -k 10 120 python -u tools/with_lib.py $PWD/dialog_amd/ab_$v.so tools/fs_walk_stats.py 4 $O/ws_$v.json > $O/ws_$v.txt 2>&1 || exit 1
  echo "$v $(grep '^[0-9]' $O/ws_$v.txt | awk '{printf "%s ", $3}')"
done
for v in a b a b; do
  timeout -k 10 200 python -u tools/with_lib.py $PWD/dialog_amd/ab_$v.so bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-extras > $O/bench_$v.json 2>/dev/null || exit 1
  echo "$v $(python3 -c "import json;d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['refit_walk_ms_per_step'])")"
done
