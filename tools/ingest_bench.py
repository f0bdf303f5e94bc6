#!/usr/bin/env python3
"""PCIe-inclusive throughput of the pinned ingest ring (surfhip_ingest_*):
1080p u8 frames already in the pinned host slots (as a decoder writing into
them would leave them) -> H2D -> detect+describe -> compacted result slab
back in pinned host memory.  Compare with bench.py's HBM-resident `value`.
Optionally the host fill of each slot (numpy copy of the frames) is timed
inside the loop too (--fill).  Prints one JSON line per depth.

    python tools/ingest_bench.py [--batch 256] [--batches 12] [--depths 1,2,3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from match_bench import load_surf  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--batches", type=int, default=12)
    ap.add_argument("--depths", default="1,2,3")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--fill", action="store_true", help="copy the frames into each slot inside the loop")
    args = ap.parse_args()
    surf = load_surf()
    surf.set_device(0)
    w, h, B = args.width, args.height, args.batch
    frames = surf.synth_frames(B, w, h)
    param = surf.make_param(4, 4.0, False, 9, 2, True, False, 4)
    # raw link rates: one pinned slot <-> HBM, synchronous copies
    det = surf.Detector(param, w, h, max_batch=B, max_pts=16384)
    ing = surf.Ingest(det, 1)
    slot = ing.acquire()
    dbuf = surf.DeviceBuffer(slot.nbytes)
    rates = {}
    for name, kind, dst, src in (("h2d", surf.H2D, dbuf.ptr, slot.ctypes.data),
                                 ("d2h", surf.D2H, slot.ctypes.data, dbuf.ptr)):
        surf.check(surf.lib.surfhip_memcpy(dst, src, slot.nbytes, kind))
        t0 = time.perf_counter()
        for _ in range(5):
            surf.check(surf.lib.surfhip_memcpy(dst, src, slot.nbytes, kind))
        rates[name + "_pinned_GBps"] = round(5 * slot.nbytes / (time.perf_counter() - t0) / 1e9, 2)
    print(json.dumps({"link": rates, "bytes": slot.nbytes}), flush=True)
    dbuf.free()
    ing.close()
    det.close()
    for depth in (int(d) for d in args.depths.split(",")):
        det = surf.Detector(param, w, h, max_batch=B, max_pts=16384)
        ing = surf.Ingest(det, depth)
        for _ in range(depth):                          # pre-fill every slot once
            ing.acquire()[:] = frames
            ing.submit(B)
        while ing.pending():
            ing.collect()
        nkp, nbytes = 0, 0
        t0 = time.perf_counter()
        for i in range(args.batches):
            if ing.pending() == depth:
                s = ing.collect(copy=False)
                nkp += int(s[4:8].view(np.int32)[0])
                nbytes += s.nbytes
            slot = ing.acquire()
            if args.fill:
                slot[:] = frames
            ing.submit(B)
        while ing.pending():
            s = ing.collect(copy=False)
            nkp += int(s[4:8].view(np.int32)[0])
            nbytes += s.nbytes
        dt = time.perf_counter() - t0
        fr = args.batches * B
        print(json.dumps({"depth": depth, "batch": B, "batches": args.batches, "fill": args.fill,
                          "frames_per_s": round(fr / dt, 1), "ms_per_batch": round(1e3 * dt / args.batches, 3),
                          "h2d_GBps": round(fr * h * surf.align_up(w, 128) / dt / 1e9, 2),
                          "d2h_GBps": round(nbytes / dt / 1e9, 2), "keypoints_per_frame": round(nkp / fr, 1)}),
              flush=True)
        ing.close()
        det.close()


if __name__ == "__main__":
    main()
