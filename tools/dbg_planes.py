#!/usr/bin/env python3
"""Debug: one frame's Hessian planes vs the oracle under the current env;
prints every differing cell (octave, scale, row, col, ref, got).
    python tools/dbg_planes.py W H NOCT FIRST"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import __graft_entry__ as ge  # noqa: E402
import oracle as orc  # noqa: E402
from test_gpu_parity import _plane_views, gpu_run  # noqa: E402

surf = ge._load_pkg()
surf.set_device(0)
w, h, noct, first = (int(a) for a in sys.argv[1:5])
frames = surf.synth_frames(1, w, h, first=first)
param = surf.make_param(noct, 4.0, upright=True)
res = gpu_run(surf, param, frames, w, h, want_ws=True, desc=False)
op = orc.make_param(noct, 4.0, upright=True)
_, ref, g, octs = orc.hessian(op, frames[0], w, h)
got = res["resp"][0]
tot = 0
for (o, s, rp), (_, _, gp) in zip(_plane_views(ref, g, octs, op), _plane_views(got, g, octs, op)):
    bad = np.argwhere(rp.view(np.uint32) != gp.view(np.uint32))
    tot += len(bad)
    for r, c in bad[:12]:
        print(f"o{o} s{s} r{r} c{c} ref {rp[r, c]!r} got {gp[r, c]!r}")
print(os.environ.get("SURFHIP_Q1"), os.environ.get("SURFHIP_FAR_STRIP"), "differing cells", tot)
