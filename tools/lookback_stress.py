"""Many in-process loopback ranks on one GPU extracting at once (every rank's single-pass selects
in flight together), repeated; one JSON line per repetition with each rank's outcome against the
one-rank run.  Tells whether the selects' look-back completes beside other contexts' spinning
selects (DLG_OPT_SEL1_TICKET=1, the default) or can give up (=0, tiles numbered by workgroup
index: DESIGN.md §6).

    python tools/lookback_stress.py W REPS [NAME=VALUE ...]     (e.g. 16 10 SEL1_TICKET=0)
"""
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dialog_amd as D  # noqa: E402
from dialog_amd.synth import SEED_BASE, plane_cloud  # noqa: E402


def main():
    W, reps = int(sys.argv[1]), int(sys.argv[2])
    opts = [(getattr(D, "DLG_OPT_" + o.split("=")[0]), int(o.split("=")[1])) for o in sys.argv[3:]]
    p, _, _ = plane_cloud(W * 4_000_000, 20, seed=SEED_BASE + 61)
    prm = D.make_params(0.02, max_iterations=4095, probability=1.0, refit_mode=D.DLG_REFIT_FAST)
    ctx = D.Context(0)
    c = D.Cloud(ctx, p)
    ref = D.extract_planes(c, prm, max_planes=20, min_inliers=500)
    c.close()
    ctx.close()
    b = [p.shape[0] * r // W for r in range(W + 1)]
    fails = 0
    for rep in range(reps):
        ctxs = D.Context.loopback_group(W, 0)
        res = [None] * W
        t0 = time.monotonic()

        def run(r):
            try:
                for o, v in opts:
                    ctxs[r].set_option(o, v)
                cl = D.Cloud(ctxs[r], p[b[r]:b[r + 1]], id_base=b[r])
                e = D.extract_planes(cl, prm, max_planes=20, min_inliers=500, capacity=p.shape[0])
                cl.close()
                ok = (e["n_planes"] == ref["n_planes"] and np.array_equal(e["inliers"], ref["inliers"])
                      and np.array_equal(e["coeffs"].view(np.uint32), ref["coeffs"].view(np.uint32)))
                res[r] = dict(ok=bool(ok), t=round(time.monotonic() - t0, 2))
            except Exception as ex:
                res[r] = dict(ok=False, err=str(ex)[:200], t=round(time.monotonic() - t0, 2))

        th = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(W)]
        [t.start() for t in th]
        for t in th:
            t.join(max(0.1, 120 - (time.monotonic() - t0)))
        hung = [r for r in range(W) if th[r].is_alive()]
        bad = [dict(rank=r, **res[r]) for r in range(W) if res[r] is None or not res[r]["ok"]]
        fails += bool(bad or hung)
        print(json.dumps(dict(rep=rep, ranks=W, opts=sys.argv[3:], hung=hung, n_ok=W - len(bad),
                              failed=bad[:3], wall_s=round(time.monotonic() - t0, 2))), flush=True)
        if hung:  # (threads stuck in the runtime: no orderly teardown)
            os._exit(3)
        for cx in ctxs:
            cx.close()
    print(json.dumps(dict(summary=True, ranks=W, reps=reps, opts=sys.argv[3:], failed_reps=fails)))


if __name__ == "__main__":
    main()
