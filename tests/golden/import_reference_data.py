"""Copy the reference's own data files into tests/golden/ (data fixtures: inputs only; the
reference holds no outputs for the RANSAC path).  Run in the build container, where
/root/reference exists; the GPU box reads only the copies.

  dataForPlane/{source,target}_plane_registration.{pcd,txt}   byte copies of
      Dialog/dataForPlane/*: polygon border vertices + per-polygon vertex counts, the format
      Registration.h:356-420 reads (11 polygons each, 1960 / 1963 vertices)
  filed_OM.npz      Dialog/result_pcd/filed_OM.pcd (147,486 points, ASCII PCD) parsed to float32
                    [N, 3] (decimal -> nearest float), stored compressed with its source SHA-256
"""
import hashlib
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from dialog_amd.pcd import read_pcd  # noqa: E402

REF = "/root/reference/Dialog"


def main():
    os.makedirs(os.path.join(HERE, "dataForPlane"), exist_ok=True)
    for side in ("source", "target"):
        for ext in ("pcd", "txt"):
            name = f"{side}_plane_registration.{ext}"
            shutil.copyfile(os.path.join(REF, "dataForPlane", name),
                            os.path.join(HERE, "dataForPlane", name))
    src = os.path.join(REF, "result_pcd", "filed_OM.pcd")
    pts = read_pcd(src)
    digest = hashlib.sha256(open(src, "rb").read()).hexdigest()
    np.savez_compressed(os.path.join(HERE, "filed_OM.npz"), points=pts, source_sha256=digest,
                        source="Dialog/result_pcd/filed_OM.pcd")
    print(pts.shape, digest)


if __name__ == "__main__":
    main()
