"""CPU: the C-ABI library builds, loads and exports every symbol include/*.h declares; without a
GPU the product fails loudly (no CPU fallback); host-only entry points behave."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import dialog_amd
from dialog_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "dialog_ransac.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dlg_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert set(syms) == set(_lib.SYMBOLS)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (dlg_\w+)", out))
    assert set(syms) <= exported


def test_library_is_gfx950_code_object():
    """The fat binary embedded in the .so carries a gfx950 code object (and no other target)."""
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


def test_params_defaults_match_pcl():
    p = dialog_amd.make_params()
    L = _lib.load()
    d = _lib.SacParams()
    L.dlg_sac_params_default(C.byref(d))
    assert d.max_iterations == 50 and d.probability == 0.99 and d.optimize == 1
    assert d.seed == 12345 and d.model == 0 and d.threshold == 0.0
    assert p.max_iterations == 50
    assert L.dlg_abi_version() == _lib.ABI_VERSION == 5
    assert L.dlg_status_string(0) == b"ok"


def test_struct_layouts_match_the_header():
    """The ctypes structs have the header's sizes (dlg_abi_struct_size reports sizeof of each): a
    binding built for another layout would read or write past the caller's struct."""
    L = _lib.load()
    pairs = [(0, _lib.Points), (1, _lib.SacParams), (2, _lib.SacStats), (3, _lib.ExtractStats),
             (4, _lib.Planes), (5, _lib.PostProcessParams)]
    for which, cls in pairs:
        assert L.dlg_abi_struct_size(which) == C.sizeof(cls), cls.__name__
    assert L.dlg_abi_struct_size(99) == -1


def test_no_device_fails_loudly(monkeypatch):
    """On a box without a gfx950 device the product refuses to run (no silent CPU path)."""
    try:
        import torch  # noqa: F401  (only to ask whether a GPU exists)
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present: covered by the -m gpu tests")
    with pytest.raises(dialog_amd.DialogError) as ei:
        dialog_amd.Context(0)
    assert ei.value.status == 3  # DLG_ERR_NO_DEVICE
    seg = dialog_amd.SACSegmentation()
    seg.setModelType(dialog_amd.SACMODEL_PLANE)
    seg.setMethodType(dialog_amd.SAC_RANSAC)
    seg.setDistanceThreshold(0.01)
    seg.setInputCloud(np.zeros((10, 3), np.float32))
    with pytest.raises(dialog_amd.DialogError):
        seg.segment()


@pytest.mark.parametrize("prog", ["shim_smoke", "plane_clouds_glue", "poly_planes_glue"])
def test_cpp_shim_compiles_and_links(tmp_path, prog):
    """The PCL-compatible C++ host shim compiles with g++ against the header and links the .so
    (shim_smoke: every shim entry; plane_clouds_glue: INTEGRATION.md §3's PlaneDetect.h adapter
    with the reference's struct Plane)."""
    src = os.path.join(ROOT, "tests", "cpp", prog + ".cpp")
    exe = tmp_path / prog
    cmd = ["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"), src, "-o", str(exe),
           "-L", os.path.dirname(_lib.LIB_PATH), "-ldialog_amd",
           f"-Wl,-rpath,{os.path.dirname(_lib.LIB_PATH)}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
