"""Polygon hand-off files of the plane stage (Dialog/PCLViewer.cpp:1341-1396 writer,
PCLViewer.cpp:1682-1791 reader): the output of the plane stage as the downstream OSnap /
HoleFilling tools read it.

    <name>.pcd              all polygon vertices (pcl::PointXYZ, ASCII), polygon after polygon
    <name>_polySize.txt     vertex count of each polygon, one per line
    <name>_polyNormal.pcd   plane normal of each polygon (pcl::Normal, ASCII; curvature 0)
    <name>_polyScale.txt    r_for_estimate_normal, once per polygon

The borders (PlaneDetect.h:1358-1440, pcl::ConcaveHull of the projected inliers, oriented so the
vertex order's right-hand normal points outward) are supplied by the caller.
"""
from __future__ import annotations

import os

import numpy as np

from .pcd import read_pcd, read_pcd_fields, write_pcd_ascii


def _stem(path: str) -> str:
    return path[:-4]  # the reference drops the last four characters (".pcd")


def write_polygons(path: str, borders, normals, scale: float) -> None:
    """borders: list of float32 [m_i, 3]; normals: [P, 3] plane normals (coeff.values[0..2])."""
    borders = [np.asarray(b, np.float32).reshape(-1, 3) for b in borders]
    normals = np.asarray(normals, np.float32).reshape(-1, 3)
    if len(borders) != normals.shape[0]:
        raise ValueError("one normal per polygon")
    verts = np.concatenate(borders, axis=0) if borders else np.zeros((0, 3), np.float32)
    write_pcd_ascii(path, verts)
    stem = _stem(path)
    with open(stem + "_polySize.txt", "w") as f:
        for b in borders:
            f.write(f"{b.shape[0]}\n")
    nrm = np.zeros((normals.shape[0], 4), np.float32)
    nrm[:, :3] = normals
    write_pcd_ascii(stem + "_polyNormal.pcd", nrm,
                    fields=("normal_x", "normal_y", "normal_z", "curvature"))
    with open(stem + "_polyScale.txt", "w") as f:
        for _ in borders:
            f.write("%g\n" % float(np.float32(scale)))  # std::ostream << float (precision 6)


def read_polygons(path: str):
    """-> (borders list of float32 [m_i, 3], normals [P, 3], scales [P])."""
    verts = read_pcd(path)
    stem = _stem(path)
    normals = read_pcd_fields(stem + "_polyNormal.pcd", ("normal_x", "normal_y", "normal_z"))
    with open(stem + "_polySize.txt") as f:
        sizes = [int(x) for x in f.read().split()]
    scales = []
    if os.path.exists(stem + "_polyScale.txt"):
        with open(stem + "_polyScale.txt") as f:
            scales = [float(x) for x in f.read().split()]
    borders, base = [], 0
    for m in sizes:
        borders.append(verts[base:base + m])
        base += m
    return borders, normals, np.asarray(scales, np.float32)


def read_polygon_pair(pcd_path: str, sizes_path: str):
    """The plane-registration polygon input (Dialog/Registration.h:356-420, files
    Dialog/dataForPlane/<side>_plane_registration.{pcd,txt}): all border vertices in one PCD and
    the vertex count of each polygon in a text file.  As the reference: counts are accumulated
    until the running sum reaches the vertex count (later entries are not read), and polygon k
    takes vertices [sum_{k-1}, sum_k).  The reference's behaviour is undefined when the counts
    overshoot the vertex count or run out before reaching it (it reads past the cloud / loops on a
    failed read): both raise ValueError here.  -> list of float32 [m_k, 3]."""
    verts = read_pcd(pcd_path)
    with open(sizes_path) as f:
        tokens = f.read().split()
    bounds, total = [], 0
    for t in tokens:
        total += int(t)
        bounds.append(total)
        if total >= verts.shape[0]:
            break
    if not bounds or bounds[-1] < verts.shape[0]:
        raise ValueError(f"{sizes_path}: polygon sizes end before the {verts.shape[0]} vertices")
    if bounds[-1] > verts.shape[0]:
        raise ValueError(f"{sizes_path}: polygon sizes overshoot the {verts.shape[0]} vertices")
    out, lo = [], 0
    for b in bounds:
        out.append(verts[lo:b].copy())
        lo = b
    return out
