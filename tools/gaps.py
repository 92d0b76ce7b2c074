"""Inter-kernel gaps of a rocprofv3 kernel trace over the last N scoring rounds:
python tools/gaps.py gpurun_out/ktr/run_kernel_trace.csv [rounds]"""
import collections
import csv
import re
import sys

r = list(csv.DictReader(open(sys.argv[1])))
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 20
r.sort(key=lambda x: int(x['Start_Timestamp']))


def nm(x):
    m = re.search(r'(k_\w+|fill\w*|copy\w*|trampoline)', x['Kernel_Name'])
    return m.group(1) if m else x['Kernel_Name'][:30]


idx = [i for i, x in enumerate(r) if 'k_score_tiles' in x['Kernel_Name']]
seg = r[idx[-rounds] - 2:]
g = collections.defaultdict(list)
for a, b in zip(seg, seg[1:]):
    g[(nm(a), nm(b))].append((int(b['Start_Timestamp']) - int(a['End_Timestamp'])) / 1e3)
busy = sum((int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e3 for x in seg)
span = (int(seg[-1]['End_Timestamp']) - int(seg[0]['Start_Timestamp'])) / 1e3
print(f"span {span:.1f} us, kernels busy {busy:.1f} us")
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[0]:22s}->{k[1]:22s} n={len(v):3d} sum={sum(v):8.1f} avg={sum(v)/len(v):7.1f}")
