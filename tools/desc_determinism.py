"""Run the config#3 batch (256 x 1080p) several times and report descriptor
bytes that differ between runs and against a max_batch=1 detector, per frame.

    python3 tools/desc_determinism.py [runs] [frames_checked_single]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from conftest import load_surf_amd  # noqa: E402

surf = load_surf_amd()

W, H, N = 1920, 1080, 256
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
nsingle = int(sys.argv[2]) if len(sys.argv) > 2 else 32
max_pts = 8192
frames = surf.synth_frames(N, W, H, first=0)
param = surf.make_param(4, 4.0, upright=True)
pitch = frames.shape[2]
det = surf.Detector(param, W, H, max_batch=N, max_pts=max_pts)
fb = surf.DeviceBuffer(frames.nbytes)
fb.upload(frames)
pb = surf.DeviceBuffer(48 * N * max_pts)
db = surf.DeviceBuffer(4 * N * max_pts * 64)
cb = surf.DeviceBuffer(4 * N)
outs = []
for r in range(runs):
    det.detect_batch(fb.ptr, N, pitch, H * pitch, pb.ptr, db.ptr, cb.ptr)
    surf.synchronize()
    counts = cb.download(np.int32, N)
    d = db.download(np.float32, N * max_pts * 64).reshape(N, max_pts, 64)
    outs.append((counts.copy(), d.copy()))
det.close()
c0, d0 = outs[0]
for r in range(1, runs):
    c, d = outs[r]
    assert (c == c0).all()
    bad = [(f, int(np.sum(np.any(d[f, :c0[f]] != d0[f, :c0[f]], axis=1)))) for f in range(N)]
    bad = [b for b in bad if b[1]]
    print(f"run {r} vs 0: frames with differing keypoints: {len(bad)} {bad[:10]}", flush=True)
    if os.environ.get("DETAIL"):
        pts = pb.download(surf.POINT_DTYPE, N * max_pts).reshape(N, max_pts)
        for f, _ in bad:
            ks = np.nonzero(np.any(d[f, :c0[f]] != d0[f, :c0[f]], axis=1))[0]
            for k in ks:
                p = pts[f, k]
                sc = 1.65 * float(p["scale"])
                step = max(int(np.rint(sc * 0.5)), 1)
                hs = int(sc)
                el = np.nonzero(d[f, k] != d0[f, k])[0]
                print(f"  f{f} k{k} x {p['x']:.1f} y {p['y']:.1f} scale {p['scale']:.3f} step {step} hs {hs} "
                      f"hmode {hs - 2 * step} maxdiff {np.max(np.abs(d[f, k] - d0[f, k])):.3g} elems {el.tolist()[:16]}")
# single-frame detector on the first frames
det1 = surf.Detector(param, W, H, max_batch=1, max_pts=max_pts)
f1 = surf.DeviceBuffer(frames[0].nbytes)
p1 = surf.DeviceBuffer(48 * max_pts)
d1 = surf.DeviceBuffer(4 * max_pts * 64)
k1 = surf.DeviceBuffer(4)
nbad = 0
for f in range(nsingle):
    f1.upload(frames[f])
    det1.detect_batch(f1.ptr, 1, pitch, 0, p1.ptr, d1.ptr, k1.ptr)
    surf.synchronize()
    n = int(k1.download(np.int32, 1)[0])
    dd = d1.download(np.float32, max_pts * 64).reshape(max_pts, 64)[:n]
    diff = np.any(dd != d0[f, :n], axis=1)
    if diff.any():
        nbad += 1
        k = int(np.argmax(diff))
        rel = float(np.max(np.abs(dd[k] - d0[f, k])))
        print(f"single vs batch frame {f}: {int(diff.sum())} keypoints differ (first {k}, max abs {rel:.3g})", flush=True)
print(f"single-frame mismatching frames: {nbad} of {nsingle}")
det1.close()
