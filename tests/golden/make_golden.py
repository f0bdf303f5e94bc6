#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ (run in the build container,
where the reference's data files exist).

Inputs: the reference's only data, /root/reference/data/left.pgm and
right.pgm (1280x960 P5), plus the 2x2-box-averaged 640x480 left image
(BASELINE config #1).  Outputs: the CPU oracle's keypoints and descriptors
(thresh 4, 4 octaves, init mask 9, sampling 2 -- main.cpp:187-204) in
canonical order.  These freeze the oracle (a restatement of the reference;
"parity unpinned" vs the CUDA binary, which cannot run here) so that any
later change to either the oracle or the HIP path is caught.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import load_oracle, load_surf_amd  # noqa: E402

DATA = "/root/reference/data"

CASES = {
    # name: (image key, upright, extend)
    "left_1280x960_upright": ("left_1280x960", True, False),
    "left_1280x960_rotated": ("left_1280x960", False, False),
    "right_1280x960_upright": ("right_1280x960", True, False),
    "left_640x480_upright": ("left_640x480", True, False),
    "left_1280x960_rotated_ext": ("left_1280x960", False, True),
}


def images(surf):
    out = {}
    for side in ("left", "right"):
        img, w, h = surf.read_pgm(os.path.join(DATA, f"{side}.pgm"), pitch=1280)
        out[f"{side}_{w}x{h}"] = img[:, :w].copy()
    left = out["left_1280x960"]
    small = surf.downsample2(left, 1280, 960)
    out["left_640x480"] = small[:, :640].copy()
    return out


def main():
    surf = load_surf_amd()
    orc = load_oracle()
    imgs = images(surf)
    np.savez_compressed(os.path.join(HERE, "images.npz"), **imgs)
    for name, (key, upright, extend) in CASES.items():
        img = imgs[key]
        h, w = img.shape
        p = orc.make_param(4, 4.0, False, 9, 2, upright, extend, 4)
        pts, desc, nc = orc.detect(p, img, w, h)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), points=pts.view(np.uint8),
                            desc=desc, meta=np.array([upright, extend, nc], np.int64),
                            image_key=np.array(key))
        print(f"{name}: {len(pts)} keypoints ({nc} candidates), octaves {np.bincount(pts['o'])}")


if __name__ == "__main__":
    main()
