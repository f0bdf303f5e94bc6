"""Probe: generic k_describe vs the oracle for several descriptor windows
(prints the worst per-keypoint L2 error and where the first bad keypoint's
descriptor differs)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "oracle")); sys.path.insert(0, os.path.join(REPO, "tests"))
import __graft_entry__ as g
surf = g._load_pkg()
import oracle as orc
from test_gpu_parity import gpu_run
surf.set_device(0)
w, h = 640, 480
frames = surf.synth_frames(1, w, h, first=40)
for wsz, ext in [(5, True), (6, True), (7, False), (7, True)]:
    for up in (True, False):
        p = surf.make_param(4, 4.0, upright=up, extend=ext, desc_wsz=wsz)
        res = gpu_run(surf, p, frames, w, h)
        op = orc.make_param(4, 4.0, upright=up, extend=ext, desc_wsz=wsz)
        o_pts, o_desc, _ = orc.detect(op, frames[0], w, h)
        gd = res["desc"][0]
        n = min(len(gd), len(o_desc))
        err = np.sqrt(((gd[:n].astype(np.float64) - o_desc[:n]) ** 2).sum(1))
        bad = np.nonzero(err > 1e-4)[0]
        msg = ""
        if len(bad):
            k = bad[0]
            diff = np.nonzero(np.abs(gd[k] - o_desc[k]) > 1e-5)[0]
            msg = f"first bad kp {k} scale {o_pts['scale'][k]:.2f} diff idx {diff[:8]} .. {diff[-3:]} ndiff {len(diff)} gpu-norm {np.linalg.norm(gd[k]):.3f}"
        print(f"wsz {wsz} ext {int(ext)} up {int(up)} nf {p.nfeatures} n {len(gd)}/{len(o_desc)} max {err.max():.3g} nbad {len(bad)} {msg}", flush=True)
