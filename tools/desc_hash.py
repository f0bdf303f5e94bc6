#!/usr/bin/env python3
"""SHA-256 of one batch's keypoints and descriptors (A/B of two builds of
libsurfhip.so that must agree bit for bit: run once per SURFHIP_LIB_DIR and
compare the lines).

    SURFHIP_LIB_DIR=cuda-surf_amd/diag/<name> python3 tools/desc_hash.py [--config5]
"""
import argparse
import hashlib
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config5", action="store_true", help="8 x 3840x2160, 5 octaves, rotated 128-D")
    ap.add_argument("--frames", type=int, default=8)
    a = ap.parse_args()
    surf = importlib.import_module("cuda-surf_amd")
    if a.config5:
        w, h, param = 3840, 2160, surf.make_param(5, 4.0, upright=False, extend=True)
        max_pts = 32768
    else:
        w, h, param = 1920, 1080, surf.make_param(4, 4.0, upright=True)
        max_pts = 8192
    n = a.frames
    frames = surf.synth_frames(n, w, h, first=11)
    pitch = frames.shape[2]
    nf = param.nfeatures
    det = surf.Detector(param, w, h, max_batch=n, max_pts=max_pts)
    fb = surf.DeviceBuffer(frames.nbytes)
    fb.upload(frames)
    pb = surf.DeviceBuffer(48 * n * max_pts)
    db = surf.DeviceBuffer(4 * n * max_pts * nf)
    cb = surf.DeviceBuffer(4 * n)
    det.detect_batch(fb.ptr, n, pitch, h * pitch, pb.ptr, db.ptr, cb.ptr)
    surf.synchronize()
    counts = cb.download(np.int32, n)
    pts = pb.download(surf.POINT_DTYPE, n * max_pts).reshape(n, max_pts)
    desc = db.download(np.float32, n * max_pts * nf).reshape(n, max_pts, nf)
    hsh = hashlib.sha256()
    for f in range(n):
        hsh.update(pts[f, :counts[f]].tobytes())
        hsh.update(desc[f, :counts[f]].tobytes())
    print(f"{os.environ.get('SURFHIP_LIB_DIR', 'default')}: keypoints {int(counts.sum())} sha256 {hsh.hexdigest()}")
    det.close()


if __name__ == "__main__":
    main()
