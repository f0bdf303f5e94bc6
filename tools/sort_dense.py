#!/usr/bin/env python3
"""Sort stage of a single dense 1080p frame (k_sort_rank with
cnt near the candidate capacity).  A uniform-noise frame gives ~10^4
candidates; the stage is timed with the detector's profiling events, rank
sort (default for <= 8 frames) against the bitonic k_sort
(SURFHIP_SORT_BITONIC, read per launch), and the keypoints of both must be
identical.

    python3 tools/sort_dense.py [thresh ...]
"""
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    surf = importlib.import_module("cuda-surf_amd")
    w, h = 1920, 1080
    pitch = surf.align_up(w, 128)
    rng = np.random.default_rng(5)
    frame = rng.integers(0, 256, size=(1, h, pitch), dtype=np.uint8)
    fb = surf.DeviceBuffer(frame.nbytes)
    fb.upload(frame)
    out = []
    for thresh in [float(a) for a in sys.argv[1:]] or [4.0, 40.0]:
        param = surf.make_param(4, thresh, upright=True)
        det = surf.Detector(param, w, h, max_batch=1, max_pts=16384)
        pb = surf.DeviceBuffer(48 * 16384)
        db = surf.DeviceBuffer(4 * 64 * 16384)
        cb = surf.DeviceBuffer(4)
        res = {"thresh": thresh}
        pts = {}
        for mode in ("rank", "bitonic"):
            if mode == "bitonic":
                os.environ["SURFHIP_SORT_BITONIC"] = "1"
            else:
                os.environ.pop("SURFHIP_SORT_BITONIC", None)
            det.set_profiling(True)
            acc = []
            for i in range(25):
                det.detect_batch(fb.ptr, 1, pitch, h * pitch, pb.ptr, db.ptr, cb.ptr)
                st = det.stage_times()
                if i >= 5:
                    acc.append(st["sort"])
            det.set_profiling(False)
            surf.synchronize()
            n = int(cb.download(np.int32, 1)[0])
            pts[mode] = pb.download(surf.POINT_DTYPE, n)
            res[f"{mode}_sort_ms"] = round(float(np.median(acc)), 4)
            res["keypoints"] = n
        res["candidates"] = int(det.candidates(1)[0])
        res["identical"] = bool(pts["rank"].tobytes() == pts["bitonic"].tobytes())
        os.environ.pop("SURFHIP_SORT_BITONIC", None)
        det.close()
        print(json.dumps(res), flush=True)
        out.append(res)
    if not all(r["identical"] for r in out):
        sys.exit(1)


if __name__ == "__main__":
    main()
