"""Build the in-tree HIP library dialog_amd/libdialog_amd.so for gfx950 (hipcc, no cmake).

Flags that matter for parity with PCL: -ffp-contract=off (no fused multiply-adds except the explicit
ones), -fhip-fp32-correctly-rounded-divide-sqrt (IEEE f32 / and sqrt), -fno-slp-vectorize (keeps
the scoring loop in single-issue f32 ops instead of v_pk_* pairs), and
-amdgpu-mfma-vgpr-form (bf16 scoring variant: MFMA accumulators in VGPRs).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libdialog_amd.so")
SOURCES = ["kernels.hip", "fsum.hip", "spatial.hip", "normals.hip", "postprocess.hip", "comm.cpp", "driver.cpp", "sac_control.cpp",
           "normals_host.cpp", "postprocess_host.cpp"]
# every header under csrc/ (a header change rebuilds every object: no per-file dependency scan)
HEADERS = sorted(f for f in os.listdir(CSRC) if f.endswith(".hpp") or f.endswith(".h"))
ARCH = os.environ.get("DLG_OFFLOAD_ARCH", "gfx950")

CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-slp-vectorize",
            "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wall", "-Wno-unused-function",
            # MFMA results in VGPRs (the VALU consumes every element; AGPR copies cost 1 op each)
            "-mllvm", "-amdgpu-mfma-vgpr-form"]
# (A/B builds only, tools/build_ab.sh: e.g. DLG_EXTRA_CXXFLAGS=-DDLG_WG_TRACE)
CXXFLAGS += os.environ.get("DLG_EXTRA_CXXFLAGS", "").split()


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(HERE, "..", "include", "dialog_ransac.h"))
    deps.append(os.path.abspath(__file__))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _compile(src: str, obj: str, verbose: bool) -> None:
    cmd = [hipcc(), f"--offload-arch={ARCH}", *CXXFLAGS, "-c", src, "-o", obj + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {os.path.basename(src)} ({r.returncode}):\n{r.stderr[-4000:]}")
    os.replace(obj + ".tmp", obj)


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile each translation unit in parallel (objects under dialog_amd/build/), then link."""
    if not force and not _stale():
        return LIB
    from concurrent.futures import ThreadPoolExecutor
    odir = os.path.join(HERE, "build")
    os.makedirs(odir, exist_ok=True)
    hdr_t = max(os.path.getmtime(d) for d in
                [os.path.join(CSRC, h) for h in HEADERS] +
                [os.path.join(HERE, "..", "include", "dialog_ransac.h"), os.path.abspath(__file__)]
                if os.path.exists(d))
    jobs = []
    objs = []
    for src in SOURCES:
        sp = os.path.join(CSRC, src)
        obj = os.path.join(odir, src + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(hdr_t, os.path.getmtime(sp)):
            jobs.append((sp, obj))
    workers = max(1, min(len(jobs), os.cpu_count() or 1, 16))
    with ThreadPoolExecutor(workers) as ex:
        for f in [ex.submit(_compile, sp, obj, verbose) for sp, obj in jobs]:
            f.result()
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", *objs, "-o", LIB + ".tmp", "-ldl", "-lpthread"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed ({r.returncode}):\n{r.stderr[-4000:]}")
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
