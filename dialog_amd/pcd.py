"""Minimal PCD v0.7 reader/writer for PointXYZ clouds (ASCII and binary).

Mirrors what the reference reads/writes: pcl::io::loadPCDFile / savePCDFileASCII on
`pcl::PointCloud<pcl::PointXYZ>` (Dialog/PCLViewer.cpp:236, Dialog/Registration.h:186-201); fields
other than x, y, z (e.g. the rgb column of Dialog/double_shadow.pcd:3) are ignored on load.
"""
from __future__ import annotations

import numpy as np

_NP = {("F", 4): np.float32, ("F", 8): np.float64, ("U", 1): np.uint8, ("U", 2): np.uint16,
       ("U", 4): np.uint32, ("I", 1): np.int8, ("I", 2): np.int16, ("I", 4): np.int32}


def read_pcd(path: str) -> np.ndarray:
    """Return float32 [N, 3] xyz."""
    with open(path, "rb") as f:
        header = {}
        while True:
            line = f.readline()
            if not line:
                raise ValueError(f"{path}: truncated PCD header")
            s = line.decode("ascii", "replace").strip()
            if not s or s.startswith("#"):
                continue
            key, _, rest = s.partition(" ")
            header[key.upper()] = rest.split()
            if key.upper() == "DATA":
                break
        body = f.read()
    fields = header["FIELDS"]
    sizes = [int(v) for v in header["SIZE"]]
    types = header["TYPE"]
    counts = [int(v) for v in header.get("COUNT", ["1"] * len(fields))]
    n = int(header["POINTS"][0])
    kind = header["DATA"][0].lower()
    cols = {}
    if kind == "ascii":
        rows = [r.split() for r in body.decode("ascii", "replace").splitlines() if r.strip()]
        rows = rows[:n]
        col = 0
        for fld, cnt in zip(fields, counts):
            if fld in ("x", "y", "z"):
                cols[fld] = np.array([float(r[col]) for r in rows], dtype=np.float32)
            col += cnt
    elif kind == "binary":
        dt = np.dtype([(f if f != "_" else f"_pad{i}", _NP[(t, s)], (c,)) if c > 1 else
                       (f if f != "_" else f"_pad{i}", _NP[(t, s)])
                       for i, (f, t, s, c) in enumerate(zip(fields, types, sizes, counts))])
        arr = np.frombuffer(body[: dt.itemsize * n], dtype=dt, count=n)
        for fld in ("x", "y", "z"):
            cols[fld] = arr[fld].astype(np.float32)
    else:
        raise ValueError(f"{path}: unsupported PCD DATA {kind}")
    return np.ascontiguousarray(np.stack([cols["x"], cols["y"], cols["z"]], axis=1))


def write_pcd_ascii(path: str, xyz: np.ndarray) -> None:
    xyz = np.asarray(xyz, np.float32)
    with open(path, "w") as f:
        f.write("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z\n"
                "SIZE 4 4 4\nTYPE F F F\nCOUNT 1 1 1\n")
        f.write(f"WIDTH {xyz.shape[0]}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\n")
        f.write(f"POINTS {xyz.shape[0]}\nDATA ascii\n")
        for p in xyz:
            f.write("%.9g %.9g %.9g\n" % (float(p[0]), float(p[1]), float(p[2])))
