#!/usr/bin/env python3
"""Which frames of a 256 x 1080p batch get a wrong fused integral image, and
where (GPU box; test infrastructure: compares with the oracle's integral).

    SURFHIP_II_FUSE=2 python3 tools/ii_batch_check.py [frames...]
"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    surf = importlib.import_module("cuda-surf_amd")
    import oracle as orc
    n, w, h = 256, 1920, 1080
    frames = surf.synth_frames(n, w, h)
    pitch = frames.shape[2]
    det = surf.Detector(surf.make_param(4, 4.0, upright=True), w, h, max_batch=n, max_pts=8192)
    print(det.hessian_kernels())
    fb = surf.DeviceBuffer(frames.nbytes)
    fb.upload(frames)
    pb = surf.DeviceBuffer(48 * n * 8192)
    cb = surf.DeviceBuffer(4 * n)
    det.detect_batch(fb.ptr, n, pitch, h * pitch, pb.ptr, None, cb.ptr)
    surf.synchronize()
    ii, iis, _, _ = det.workspace()
    ip = surf.align_up(w + 1, 128)
    sel = [int(a) for a in sys.argv[1:]] or range(n)
    nbad = 0
    for f in sel:
        got = surf.download_ptr(ii + 4 * f * iis, np.int32, (h + 1) * ip).reshape(h + 1, ip)
        bad = np.argwhere(got != orc.integral(frames[f], w, h))
        if len(bad):
            nbad += 1
            rows = np.unique(bad[:, 0])
            print(f"frame {f}: {len(bad)} values differ, rows {rows[:8].tolist()}, "
                  f"columns {bad[:, 1].min()}-{bad[:, 1].max()}", flush=True)
    print(f"{nbad} of {len(sel)} frames differ")
    det.close()


if __name__ == "__main__":
    main()
