"""The C++ drop-in on the GPU: cuda-surf_amd/surf_demo (tools/surf_demo.cpp,
the reference's main.cpp:163-283 flow -- initDevice, cudaMallocPitch,
cudaMemcpy2D, Surfor::init, detectAndCompute x2, match -- compiled against
include/surf.h + cuda_utils.h and linked to libsurf.so) on the reference's own
left/right images, its dumps compared with the committed golden fixtures."""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

from conftest import REPO, assert_points_equal, desc_l2
from test_gpu_parity import DESC_TOL, GOLDEN, MATCH_FIELDS, assert_match_equal

pytestmark = pytest.mark.gpu
DEMO = os.path.join(REPO, "cuda-surf_amd", "surf_demo")


def _read_dump(path, dtype):
    b = np.fromfile(path, np.uint8)
    n, nf = (int(v) for v in b[:8].view(np.int32))
    pts = b[8:8 + 48 * n].view(dtype)
    desc = b[8 + 48 * n:].view(np.float32).reshape(n, nf) if nf else None
    return pts, desc


def test_surf_demo_left_right_vs_golden(surf, orc, tmp_path):
    assert os.path.exists(DEMO), "build with make -C cuda-surf_amd (surf_demo)"
    imgs = np.load(os.path.join(GOLDEN, "images.npz"))
    paths = []
    for side in ("left", "right"):
        img = imgs[f"{side}_1280x960"]
        p = tmp_path / f"{side}.pgm"
        with open(p, "wb") as fh:
            fh.write(b"P5\n1280 960\n255\n" + np.ascontiguousarray(img).tobytes())
        paths.append(str(p))
    prefix = str(tmp_path / "out")
    r = subprocess.run([DEMO, "0", paths[0], paths[1], "3", prefix], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "Number of features1: 2739" in r.stdout, r.stdout
    got = {}
    for side in ("left", "right"):
        pts, desc = _read_dump(f"{prefix}_{side}.bin", surf.POINT_DTYPE)
        z = np.load(os.path.join(GOLDEN, f"{side}_1280x960_upright.npz"))
        ref = z["points"].view(surf.POINT_DTYPE)
        assert len(pts) == len(ref), side
        assert_points_equal(pts, ref)
        assert desc_l2(desc, z["desc"]).max() <= DESC_TOL, side
        got[side] = (pts, desc)
    m, _ = _read_dump(f"{prefix}_match.bin", surf.POINT_DTYPE)
    # match on the GPU's own descriptors is bit-exact with the oracle's
    # findMaxCorr (reference tile-tail behaviour, flags 0) ...
    ref = orc.match(got["left"][0], got["right"][0], got["left"][1], got["right"][1])
    assert_match_equal(m, ref)
    # ... and agrees with the frozen golden match where the best is clear
    zm = np.load(os.path.join(GOLDEN, "match_left_right_upright.npz"))
    clear = zm["ref_ambiguity"] < 0.99
    assert (m["match"][clear] == zm["ref_match"][clear]).mean() > 0.99
    for f in MATCH_FIELDS:
        assert len(m[f]) == len(zm[f"ref_{f}"])
