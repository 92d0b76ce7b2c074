"""Per-launch HBM traffic of the dominant kernels from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
runs of `bench.py --steps 1 --warmup 0` (separate passes, as MI355X_MICROARCH.md prescribes).

FETCH_SIZE/WRITE_SIZE are in KB (1024 B).  gfx950 counts exactly half of the bytes of a wide
(16 B/lane) coalesced read; other widths are uncalibrated (MI355X_MICROARCH.md: calibrate on a
known byte count in your own access pattern), so the factor for our 4-B/lane SoA reads is
measured here on k_absmax, which reads x, y, z of every uploaded point exactly once (12 B per
point, the same 4-B/lane pattern as the scoring kernel's point loads).  Writes ->
profiles/score_traffic.json.
"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(path, counter):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        if not m:
            continue
        out[m.group(1)].append((int(r["Dispatch_Id"]), float(r["Counter_Value"]), int(r["Grid_Size"])))
    return out


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE") if len(sys.argv) > 2 else {}
    bench = None
    if len(sys.argv) > 3:  # the bench JSON line (possibly inside a log with other output)
        lines = [ln for ln in open(sys.argv[3]).read().splitlines() if ln.startswith("{")]
        bench = json.loads(lines[-1])
    res = {}
    for k, rows in fetch.items():
        vals = [v for _, v, _ in rows]
        res[k] = {"launches": len(rows), "fetch_bytes_mean": 1024 * sum(vals) / len(vals)}
        if k in write:
            w = [v for _, v, _ in write[k]]
            res[k]["write_bytes_mean"] = 1024 * sum(w) / len(w)
    # calibration on k_absmax (upload: 12 B per point, read once, 4-B lane loads)
    ab = sorted(fetch.get("k_absmax", []))
    cal = None
    if ab and bench:
        cal = (12.0 * bench["config"]["points_per_gpu"]) / (1024 * ab[0][1])
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), bench.py --steps 1 "
                     "--warmup 0; reads x calibration (k_absmax: 12 B/point)",
           "kernels": res, "read_calibration_dword_loads": cal}
    # one scoring launch = k_prune_supers + k_score_tiles (pruned, default), else the exhaustive kernel
    keys = [k for k in ("k_prune_supers", "k_score_tiles_ex", "k_score_tiles_rl", "k_score_tiles") if k in res][:2] or \
           (["k_score_bf16"] if "k_score_bf16" in res else ["k_score"])
    if all(k in res for k in keys) and cal:
        out["kernel"] = " + ".join(keys)
        out["hbm_bytes_per_launch"] = sum(res[k]["fetch_bytes_mean"] * cal + res[k].get("write_bytes_mean", 0.0)
                                          for k in keys)
    json.dump(out, open(os.path.join(ROOT, "profiles", "score_traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
