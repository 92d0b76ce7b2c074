"""A/B of the scoring-kernel variants on the GPU (one process, interleaved rounds, counts checked
equal across variants).  Usage: python tools/score_ab.py [n_points] [D] [rounds]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes as C  # noqa: E402

import dialog_amd as D  # noqa: E402
from dialog_amd import _lib  # noqa: E402
from dialog_amd.synth import SEED_BASE, plane_cloud  # noqa: E402

NAMES = {0: "exact_p8", 1: "band_p8", 2: "min3_p8", 3: "exact_p16", 4: "min3_p16", 5: "exact_p4",
         6: "min3_p4", 7: "exactS_p8g8", 8: "min3S_p8g8", 9: "exactS_p4g8", 10: "exactS_p8g4",
         11: "mfma_pa32", 12: "mfma_pa16", 13: "mfma_pa8", 14: "lanes_exact", 15: "lanes_min3",
         16: "lds_exact", 17: "lds_min3", 18: "bf16_t4", 19: "bf16_t8", 20: "pruned"}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    nh = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    variants = [int(v) for v in os.environ.get("VARIANTS", "0,5,12,16,17").split(",")]
    pts, _, _ = plane_cloud(n, 20, seed=SEED_BASE + 3, shard=0)
    ctx = D.Context(0)
    cloud = D.Cloud(ctx, pts)
    L = _lib.load()
    res = {v: [] for v in variants}
    ref = None
    for r in range(rounds):
        for v in variants:
            ms = C.c_double()
            cnt = np.zeros(nh, np.int32)
            ctx.check(L.dlg_score_benchmark(ctx.h, cloud.h, nh, v, 3, 0.02, C.byref(ms),
                                            cnt.ctypes.data_as(C.POINTER(C.c_int32))))
            res[v].append(ms.value)
            if ref is None:
                ref = cnt.copy()
            if not os.environ.get("SCORE_AB_NOCHECK"):
                assert np.array_equal(cnt, ref), f"variant {v} counts differ"
            elif not np.array_equal(cnt, ref):
                print(f"variant {v}: {int((cnt != ref).sum())} counts differ", file=sys.stderr)
    out = {}
    for v in variants:
        med = float(np.median(res[v]))
        tps = n * nh / (med / 1e3)
        out[NAMES[v]] = dict(ms_median=round(med, 4), ms_min=round(min(res[v]), 4),
                             T_tests_per_s=round(tps / 1e12, 3))
    print(json.dumps(dict(n=n, D=nh, rounds=rounds, counts_equal=True, total_inliers=int(ref.sum()),
                          variants=out), indent=1))


if __name__ == "__main__":
    main()
