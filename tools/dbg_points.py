#!/usr/bin/env python3
"""Debug: GPU vs oracle keypoints for one parameter set; prints per-octave
counts and the first differing keypoints.
    python tools/dbg_points.py INIT_MASK [W H NOCT THRESH DOUBLED]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
os.environ.setdefault("SURFHIP_HESS_GATHER", "0")
from conftest import load_oracle, load_surf_amd  # noqa: E402

surf, orc = load_surf_amd(), load_oracle()
a = sys.argv[1:]
init = int(a[0])
w, h, noct = (int(a[1]), int(a[2]), int(a[3])) if len(a) > 3 else (640, 480, 4)
thresh = float(a[4]) if len(a) > 4 else 2.0
dbl = len(a) > 5 and a[5] == "1"
sys.path.insert(0, os.path.join(REPO, "tests"))
from test_gpu_parity import gpu_run  # noqa: E402

frames = surf.synth_frames(1, w, h, first=90)
param = surf.make_param(noct, thresh, doubled=dbl, init_mask_size=init, upright=True)
res = gpu_run(surf, param, frames, w, h, want_ws=True)
op = orc.make_param(noct, thresh, dbl, init, 2, True, False, 4)
o_pts, o_desc, nc = orc.detect(op, frames[0], w, h)
g = res["pts"][0]
print("max_scale", param.max_scale, "cand gpu", res["cand"][0], "oracle", nc, "pts gpu", len(g), "oracle", len(o_pts))
for o in range(noct):
    print(" octave", o, "gpu", int((g["o"] == o).sum()), "oracle", int((o_pts["o"] == o).sum()))
n = min(len(g), len(o_pts))
for i in range(n):
    if (g[i]["x"], g[i]["y"], g[i]["scale"]) != (o_pts[i]["x"], o_pts[i]["y"], o_pts[i]["scale"]):
        print(" first diff at", i)
        for j in range(max(0, i - 2), min(n, i + 6)):
            print("  gpu", g[j][["o", "x", "y", "scale", "strength"]], " ora", o_pts[j][["o", "x", "y", "scale", "strength"]])
        break
