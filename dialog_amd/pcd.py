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


def read_pcd_fields(path: str, fields) -> np.ndarray:
    """Named float fields (e.g. normal_x normal_y normal_z curvature) as float32 [N, len(fields)]."""
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
    names = header["FIELDS"]
    counts = [int(v) for v in header.get("COUNT", ["1"] * len(names))]
    n = int(header["POINTS"][0])
    if header["DATA"][0].lower() != "ascii":
        raise ValueError(f"{path}: read_pcd_fields reads ASCII PCD only")
    rows = [r.split() for r in body.decode("ascii", "replace").splitlines() if r.strip()][:n]
    pos, col = {}, 0
    for fld, cnt in zip(names, counts):
        pos[fld] = col
        col += cnt
    out = np.empty((len(rows), len(fields)), np.float32)
    for k, fld in enumerate(fields):
        out[:, k] = [float(r[pos[fld]]) for r in rows]
    return out


def write_pcd_ascii(path: str, data: np.ndarray, fields=("x", "y", "z"), precision: int = 8) -> None:
    """pcl::io::savePCDFileASCII: v0.7 header, one line per point, floats printed as an ostream
    with precision(8) prints them (%g style; nan/inf as 'nan'/'inf')."""
    data = np.asarray(data, np.float32).reshape(-1, len(fields))
    n = data.shape[0]
    k = len(fields)
    with open(path, "w") as f:
        f.write("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\n")
        f.write("FIELDS " + " ".join(fields) + "\n")
        f.write("SIZE " + " ".join(["4"] * k) + "\nTYPE " + " ".join(["F"] * k) + "\n")
        f.write("COUNT " + " ".join(["1"] * k) + "\n")
        f.write(f"WIDTH {n}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {n}\nDATA ascii\n")
        fmt = " ".join([f"%.{precision}g"] * k) + "\n"
        for row in data:
            f.write(fmt % tuple(float(v) for v in row))
