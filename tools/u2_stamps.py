#!/usr/bin/env python3
"""(diagnostic) Where k_describe_u2's time goes per keypoint: runs the bench
batch's detect_batch a few times on a SURF_DIAG_U2_STAMP build
(SURFHIP_LIB_DIR=cuda-surf_amd/diag/<name>) and prints the s_memtime ticks
per keypoint of each phase (setup, rows by path, reduction, normalise+store),
summed over all waves of the last launch, and the keypoints per row path.
    SURFHIP_LIB_DIR=cuda-surf_amd/diag/ust python3 tools/u2_stamps.py"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402,F401
import bench  # noqa: E402

surf = bench.load_surf()
W, H, B = 1920, 1080, 256
pitch = surf.align_up(W, 128)
frames = surf.synth_frames(B, W, H, pitch)
buf = surf.DeviceBuffer(frames.nbytes)
buf.upload(frames)
param = surf.make_param(4, 4.0, False, 9, 2, True, False, 4)
mp = 65536
det = surf.Detector(param, W, H, max_batch=B, max_pts=mp)
pb = surf.DeviceBuffer(48 * B * mp)
db = surf.DeviceBuffer(4 * B * mp * 64)
cb = surf.DeviceBuffer(4 * B)
for _ in range(4):
    det.detect_batch(buf.ptr, B, pitch, H * pitch, pb.ptr, db.ptr, cb.ptr)
surf.synchronize()
lib = C.CDLL(os.path.join(os.environ["SURFHIP_LIB_DIR"], "libsurfhip.so"))
st = np.zeros((8192, 12), np.uint64)
assert lib.surfhip_diag_u2_stamps(st.ctypes.data_as(C.c_void_p)) == 0
st = st.astype(np.float64)
tot = st.sum(axis=0)
n = tot[6] + tot[7] + tot[8]
names = ["setup", "rows seg", "rows sparse", "rows generic", "reduction", "norm+store"]
print(f"keypoints {int(n)}: seg {int(tot[6])} sparse {int(tot[7])} generic {int(tot[8])}")
allt = tot[:6].sum()
for i, nm in enumerate(names):
    per = tot[i] / max(1, (tot[5 + i] if 1 <= i <= 3 else n))
    print(f"{nm:13s} {tot[i] / allt * 100:5.1f} %   {per:9.1f} ticks per keypoint (of its kind)")
print(f"all phases {allt / n:.1f} ticks per keypoint per wave")
print(f"seg: first ring wait {tot[9] / max(1, tot[6]):.1f} ticks per keypoint; narrow (W4 <= 16) "
      f"{int(tot[10])} keypoints, rows {tot[11] / max(1, tot[10]):.1f} ticks; wide "
      f"{int(tot[6] - tot[10])}, rows {(tot[1] - tot[11]) / max(1, tot[6] - tot[10]):.1f} ticks")
