"""C4's 100M-point cloud over 8 in-process loopback ranks (tests/test_fullsize_golden.py's
sharded run), repeated, with context options given on the command line; one JSON line per run:
every rank's outcome (ok + bits equal to the golden ones, or its error) and wall time; with
PROFILE=1 also every rank's phase split (score / select / PCL refit walk / rebase / repair ms).

    python tools/c4_loopback_diag.py pcl 3 FS_ONE_WALK=1 SEL1_TICKET=0 BOUNDS_STREAM=1

Used to tell a hang's cause apart: with the group abort, a rank that fails no
longer leaves its peers waiting -- every rank returns, and the failing rank's error is printed.
"""
import hashlib
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dialog_amd as D  # noqa: E402
from dialog_amd.synth import plane_cloud  # noqa: E402

DB = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    mode, reps = sys.argv[1], int(sys.argv[2])
    opts = [(getattr(D, "DLG_OPT_" + o.split("=")[0]), int(o.split("=")[1])) for o in sys.argv[3:]]
    prof = os.environ.get("PROFILE") == "1"
    w = DB["c4shape"]
    g = w["modes"][mode]
    p, _, _ = plane_cloud(w["n_points"], w["planes"], seed=w["seed"], shares=w["shares"])
    W = 8
    b = [p.shape[0] * r // W for r in range(W + 1)]
    prm = D.make_params(0.02, max_iterations=4095, probability=1.0, hypotheses_per_launch=4096,
                        refit_mode=D.DLG_REFIT_PCL if mode == "pcl" else D.DLG_REFIT_FAST)
    for rep in range(reps):
        ctxs = D.Context.loopback_group(W, 0)
        res = [None] * W
        t0 = time.monotonic()

        def run(r):
            try:
                for o, v in opts:
                    ctxs[r].set_option(o, v)
                if prof:
                    ctxs[r].set_profiling(True)
                c = D.Cloud(ctxs[r], p[b[r]:b[r + 1]], id_base=b[r])
                e = D.extract_planes(c, prm, max_planes=20, min_inliers=500, capacity=p.shape[0])
                c.close()
                offs = e["offsets"]
                ok = ([[int(v) for v in cc.view(np.uint32)] for cc in e["coeffs"]] == g["coeff_bits"]
                      and [sha(e["inliers"][offs[k]:offs[k + 1]]) for k in range(e["n_planes"])]
                      == g["inliers_sha256"])
                res[r] = dict(rank=r, ok=bool(ok), t=round(time.monotonic() - t0, 2))
                if prof:
                    st = e["stats"]
                    res[r]["ms"] = {k: round(st[k], 3) for k in (
                        "score_ms", "select_ms", "refit_walk_ms", "refit_rebase_ms",
                        "refit_repair_ms", "wall_ms")}
                    res[r]["rounds"] = st["rounds"]
            except Exception as ex:
                res[r] = dict(rank=r, ok=False, err=str(ex), t=round(time.monotonic() - t0, 2))

        th = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(W)]
        [t.start() for t in th]
        for t in th:
            t.join(max(0.1, 200 - (time.monotonic() - t0)))
        hung = [r for r in range(W) if th[r].is_alive()]
        print(json.dumps(dict(rep=rep, mode=mode, opts=sys.argv[3:], hung=hung, ranks=res)),
              flush=True)
        if hung:  # (threads stuck in the runtime: no orderly teardown)
            os._exit(3)
        for c in ctxs:
            c.close()


if __name__ == "__main__":
    main()
