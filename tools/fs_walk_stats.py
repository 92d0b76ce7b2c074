"""Walk counters of DLG_REFIT_PCL's device sums on the C3 planes' inliers (dlg_float_sums)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dialog_amd as D  # noqa: E402
from dialog_amd.synth import plane_cloud  # noqa: E402

ctx = D.Context(0)
p, lab, planes = plane_cloud(10_000_000, 20, seed=0xD1A106 + 3)
out = []
for k in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
    xyz = np.ascontiguousarray(p[lab == k])
    sums, co, unc, ms, ws = ctx.float_sums(xyz, cin=planes[k], reps=3, walk_stats=True)
    out.append({"plane": k, "n": int(xyz.shape[0]), "ms": round(ms, 4),
                "chains": ws.tolist()})
    print(k, xyz.shape[0], round(ms, 4), "walked/pass/slow/step/rerun/clk/clk_step/summary/"
          "table/miss_none/miss_range/miss_mask per chain:", flush=True)
    for c in range(9):
        w = [int(v) for v in ws[c].tolist()]
        lo = [v & 0xFFFFFFFF for v in w]
        lh = [(w[3] >> (24 + 8 * b)) & 0xFF for b in range(5)]
        print("   ", [lo[0], lo[1], lo[2], w[3] & 0xFFFFFF, lo[4], w[5], w[6], lo[7], w[7] >> 32,
                      w[1] >> 32, w[2] >> 32, w[4] >> 32], "|lead| <128/<512/<4096/more/inexact:",
              lh, flush=True)
json.dump(out, open(sys.argv[2] if len(sys.argv) > 2 else "/dev/null", "w"))
