"""PCD and polygon hand-off file I/O (host side of the plane stage's output;
Dialog/PCLViewer.cpp:1341-1396 writer, :1682-1791 reader)."""
import os

import numpy as np

from dialog_amd.pcd import read_pcd, read_pcd_fields, write_pcd_ascii
from dialog_amd.polyio import read_polygons, write_polygons

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_pcd_ascii_roundtrip_and_header(tmp_path):
    rng = np.random.default_rng(0)
    p = rng.normal(size=(100, 3)).astype(np.float32) * 10
    p[3] = [np.nan, 1e-5, -2.5]
    path = str(tmp_path / "c.pcd")
    write_pcd_ascii(path, p)
    lines = open(path).read().splitlines()
    assert lines[:11] == ["# .PCD v0.7 - Point Cloud Data file format", "VERSION 0.7",
                          "FIELDS x y z", "SIZE 4 4 4", "TYPE F F F", "COUNT 1 1 1", "WIDTH 100",
                          "HEIGHT 1", "VIEWPOINT 0 0 0 1 0 0 0", "POINTS 100", "DATA ascii"]
    assert lines[14] == "nan 9.9999997e-06 -2.5"  # float(1e-5) at ostream precision 8
    q = read_pcd(path)
    ok = ~np.isnan(p).any(1)
    # precision 8 (PCL's default): relative error below 1e-7
    np.testing.assert_allclose(q[ok], p[ok], rtol=1e-7, atol=0)


def test_reference_pcd_reads():
    p = read_pcd(os.path.join(GOLDEN, "double_shadow.pcd"))
    assert p.shape == (991, 3) and np.isfinite(p).all()


def test_polygon_files_roundtrip(tmp_path):
    b1 = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0]], np.float32)
    b2 = np.array([[0, 0, 1], [2, 0, 1], [0, 2, 1]], np.float32)
    nrm = np.array([[0, 0, 1], [0, 0, -1]], np.float32)
    path = str(tmp_path / "planes.pcd")
    write_polygons(path, [b1, b2], nrm, 0.5)
    for suffix in ("_polySize.txt", "_polyNormal.pcd", "_polyScale.txt"):
        assert os.path.exists(str(tmp_path / "planes") + suffix)
    assert open(str(tmp_path / "planes_polySize.txt")).read() == "4\n3\n"
    assert open(str(tmp_path / "planes_polyScale.txt")).read() == "0.5\n0.5\n"
    borders, normals, scales = read_polygons(path)
    assert len(borders) == 2
    np.testing.assert_array_equal(borders[0], b1)
    np.testing.assert_array_equal(borders[1], b2)
    np.testing.assert_array_equal(normals, nrm)
    np.testing.assert_array_equal(scales, [0.5, 0.5])
    n4 = read_pcd_fields(str(tmp_path / "planes_polyNormal.pcd"),
                         ("normal_x", "normal_y", "normal_z", "curvature"))
    assert np.all(n4[:, 3] == 0)
