"""A/B of the scoring kernels on the GPU (one process, interleaved rounds, counts checked equal
across kernels).  Usage: python tools/score_ab.py [n_points] [D] [rounds]
KERNELS=0,1,2,... (DLG_SCORE_EXACT, DLG_SCORE_BF16, DLG_SCORE_PRUNED with the tile scorer of
TILE_OPT: 2 lanes-as-planes exact (default), 3 bf16 blocks, 5-6 A/B variants); PRUNE_STATS=1 also prints the
pruned kernel's work counters per launch (dlg_prune_stats).  The round-1 A/B of the retired
variants (FMA prefilters, scalar coefficients, f32 MFMA, lanes-as-planes) is recorded in
profiles/r01_score_variants_ab.json and DESIGN.md."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes as C  # noqa: E402

import dialog_amd as D  # noqa: E402
from dialog_amd import _lib  # noqa: E402
from dialog_amd.synth import SEED_BASE, plane_cloud  # noqa: E402

NAMES = {0: "exact_p4", 1: "bf16_t8", 2: "pruned_ex", 3: "pruned_bf16", 5: "pruned_ex_k1",
         6: "pruned_ex_k4", 7: "pruned_ex_pk", 8: "pruned_mfma", 9: "pruned_ex_claim_r4",
         10: "pruned_ex_claim_class", 11: "pruned_ex_claim_tail"}
# DLG_OPT_PRUNE_TILE_SCORER per pruned variant (2: DLG_TILE_EXACT, the default; 11, 12, 14: A/B
# only)
TILE_OPT = {2: 0, 3: 1, 5: 11, 6: 14, 7: 12, 8: 2, 9: 15, 10: 16, 11: 17}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    nh = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    variants = [int(v) for v in os.environ.get("KERNELS", "2,3").split(",")]
    want_stats = os.environ.get("PRUNE_STATS") == "1"
    pts, _, _ = plane_cloud(n, 20, seed=SEED_BASE + 3, shard=0)
    ctx = D.Context(0)
    if want_stats:
        ctx.set_option(D.DLG_OPT_PRUNE_STATS, 1)
    cloud = D.Cloud(ctx, pts)
    L = _lib.load()
    res = {v: [] for v in variants}
    ref = None
    for r in range(rounds):
        for v in variants:
            ms = C.c_double()
            cnt = np.zeros(nh, np.int32)
            ctx.set_option(D.DLG_OPT_PRUNE_TILE_SCORER, TILE_OPT.get(v, D.DLG_TILE_EXACT))
            ctx.check(L.dlg_score_benchmark(ctx.h, cloud.h, nh, min(v, 2), 3, 0.02, C.byref(ms),
                                            cnt.ctypes.data_as(C.POINTER(C.c_int32))))
            res[v].append(ms.value)
            if ref is None:
                ref = cnt.copy()
            assert np.array_equal(cnt, ref), f"kernel {v} counts differ"
    out = {}
    for v in variants:
        med = float(np.median(res[v]))
        tps = n * nh / (med / 1e3)
        out[NAMES[v]] = dict(ms_median=round(med, 4), ms_min=round(min(res[v]), 4),
                             T_tests_per_s=round(tps / 1e12, 3))
    extra = {}
    if want_stats:
        st = ctx.prune_stats(reset=True)
        launches = rounds * 3 * sum(v >= 2 for v in variants)
        if launches:
            extra["pruned_per_launch"] = {k: v / launches for k, v in st.items()}
            extra["pruned_per_launch"]["pair_fraction"] = st["pairs"] / launches / (n * nh / 32)
            if st["workgroups"]:  # (100 MHz ticks: the workgroups' spans against the longest)
                extra["wg_span_us_mean"] = st["wg_ticks_sum"] / st["workgroups"] / 100.0
                extra["wg_span_us_max"] = st["wg_ticks_max"] / 100.0
    print(json.dumps(dict(n=n, D=nh, rounds=rounds, counts_equal=True, total_inliers=int(ref.sum()),
                          kernels=out, **extra), indent=1))


if __name__ == "__main__":
    main()
