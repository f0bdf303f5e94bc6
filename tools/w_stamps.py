#!/usr/bin/env python3
"""(diagnostic) Barrier timeline of one k_hess_w workgroup: run the Hessian
of the bench batch several times on a SURF_DIAG_W_STAMP build
(SURFHIP_LIB_DIR=cuda-surf_amd/diag/<name>), read the s_memtime stamps every
wave took before / after each barrier (surfhip_diag_w_stamps) and print, per
wave role, the mean work time between barriers, the mean wait at them and
how often that wave arrived last.
    SURFHIP_LIB_DIR=cuda-surf_amd/diag/wst python3 tools/w_stamps.py"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402,F401  (one HIP runtime in the process)
import bench  # noqa: E402

surf = bench.load_surf()
W, H, B = 1920, 1080, 256
pitch = surf.align_up(W, 128)
frames = surf.synth_frames(B, W, H, pitch)
buf = surf.DeviceBuffer(frames.nbytes)
buf.upload(frames)
param = surf.make_param(4, 4.0, False, 9, 2, True, False, 4)
det = surf.Detector(param, W, H, max_batch=B, max_pts=65536)
det.run_integral(buf.ptr, B, pitch, H * pitch)
for _ in range(12):
    det.run_hessian(B)
surf.synchronize()
lib = C.CDLL(os.path.join(os.environ["SURFHIP_LIB_DIR"], "libsurfhip.so"))
st = np.zeros((16, 400, 2), np.uint64)
assert lib.surfhip_diag_w_stamps(st.ctypes.data_as(C.c_void_p)) == 0
st = st.astype(np.int64)
roles = ["prod0", "prod1", "prod2", "o1s0a", "o1s0b", "o1s1a", "o1s1b", "o1s2a", "o1s2b", "o2s0", "o2s1", "o2s2",
         "o3s0", "o3s1", "o3s2"]
n = int((st[:15, :, 1] > 0).all(axis=0).sum())
arr, lv = st[:15, :n, 0], st[:15, :n, 1]
np.save(os.path.join(REPO, "gpurun_out", "w_stamps.npy"), st)
# one launch: the stamps between two launch gaps (an interval far above the median)
iv = np.diff(lv.max(axis=0))
med = np.median(iv)
gaps = [0] + [i + 1 for i in np.nonzero((iv > 20 * med) | (iv < 0))[0]] + [n]
a, b = max(zip(gaps[:-1], gaps[1:]), key=lambda t: t[1] - t[0])
arr, lv = arr[:, a:b], lv[:, a:b]
last = np.argmax(arr, axis=0)
out = {"barriers_in_launch": int(b - a)}
for w, r in enumerate(roles):
    work = arr[w, 1:] - lv[w, :-1]
    wait = lv[w, :] - arr[w, :]
    out[r] = {"work_mean": float(work.mean()), "wait_mean": float(wait.mean()), "last_arrivals": int((last == w).sum())}
    print(f"{r:6s} work {work.mean():8.1f}  wait {wait.mean():8.1f}  last {int((last == w).sum()):4d}")
iv = np.diff(lv.max(axis=0))
print(f"barriers {b - a} in one launch, interval mean {iv.mean():.1f} ticks (median {np.median(iv):.1f}), "
      f"launch {lv.max() - arr.min()} ticks")
out["interval_mean"] = float(iv.mean())
json.dump(out, open(os.path.join(REPO, "gpurun_out", "w_stamps.json"), "w"), indent=1)
