#!/usr/bin/env python3
"""Generate tests/golden/match_left_right_upright.npz: Surfor::match of the
left against the right 1280x960 image (main.cpp:250 matches exactly this
pair), computed by the CPU oracle's findMaxCorr restatement (or_match) from
the committed keypoint/descriptor fixtures of make_golden.py.  Both the
reference's tile-tail behaviour (surfd.cu:2569 drops the last partial tile of
set 2) and the full-tail option are frozen.  Needs no reference files.

    python tests/golden/make_golden_match.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import load_oracle  # noqa: E402

FIELDS = ("score", "match", "match_x", "match_y", "ambiguity")


def load(name, orc):
    z = np.load(os.path.join(HERE, name + ".npz"))
    return z["points"].view(orc.POINT_DTYPE), z["desc"]


def main():
    orc = load_oracle()
    p1, f1 = load("left_1280x960_upright", orc)
    p2, f2 = load("right_1280x960_upright", orc)
    out = {}
    for tag, full in (("ref", False), ("full", True)):
        m = orc.match(p1, p2, f1, f2, full_tail=full)
        for f in FIELDS:
            out[f"{tag}_{f}"] = m[f]
    np.savez_compressed(os.path.join(HERE, "match_left_right_upright.npz"), **out)
    print("n1", len(p1), "n2", len(p2), "matched", int((out["ref_match"] >= 0).sum()))


if __name__ == "__main__":
    main()
