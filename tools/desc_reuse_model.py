#!/usr/bin/env python3
"""Model of the upright describe's integral reads, per keypoint against
shared tiles ("row reuse across neighbouring keypoints").
CPU only: one synthetic 1920x1080 frame of the headline batch, keypoints from
the oracle (config #3: 4 octaves, thresh 4, upright 64-D), window geometry as
k_describe_u2 derives it (surfd.cu:1566-1615 via DESIGN §Descriptor).

Per keypoint, k_describe_u2 DMAs the integral rows r, r + 1 of its valid grid
rows plus two grid rows either side (the Haar terms' rows r - s / r + s + 1),
each as its column span of W4 16-B chunks.  A shared-tile design must instead
hold, for the keypoints whose centres fall in a T x T core, the bounding box
of their windows (rows x columns, any row a keypoint of step 1 needs) -- in
LDS, 160 KiB per CU.  The script prints both byte counts per frame.

    python3 tools/desc_reuse_model.py [--frame 0]
"""
from __future__ import annotations

import argparse
import math
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def rn(x: float) -> int:
    return int(np.rint(np.float32(x)))


def window(p):
    """k_describe_u2's row set and column span of one keypoint (wsz 4)."""
    scale = np.float32(1.65) * np.float32(p["scale"])
    step = max(rn(scale * np.float32(0.5)), 1)
    ix, iy = rn(p["x"]), rn(p["y"])
    dy0 = np.float32(p["y"]) - np.float32(iy)
    spacing = scale * np.float32(3.0)
    iradius = rn(np.float32(spacing * np.float32(5.0) * np.float32(0.5)) / np.float32(step))
    side = 2 * iradius + 1
    ts = [t for t in range(side)
          if -1.0 < (np.float32(step * (t - iradius)) - dy0) / spacing + np.float32(1.5) < 4.0]
    t0, nv = (ts[0], len(ts)) if ts else (0, 0)
    rows = set()
    for t in range(t0 - 2, t0 + nv + 2):
        r = iy + (t - iradius) * step
        rows.update((r, r + 1))
    cs = (ix + (-2 - iradius) * step) & ~3
    w4 = (ix + (side + 1 - iradius) * step + 2 - cs + 3) >> 2
    return step, ix, iy, rows, cs, w4


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--frame", type=int, default=0)
    args = ap.parse_args()
    import oracle
    import importlib
    surf = importlib.import_module("cuda-surf_amd")  # synthetic frames only (host code)
    W, H = 1920, 1080
    img = surf.synth_frames(1, W, H, first=args.frame)[0]
    prm = oracle.make_param(4, 4.0, False, 9, 2, True, False, 4)
    pts, _, _ = oracle.detect(prm, img, W, H, desc=False)
    n = len(pts)
    win = [window(p) for p in pts]
    per_kp = sum(len(rows) * w4 * 16 for _, _, _, rows, _, w4 in win)
    ii_bytes = 1921 * 1081 * 4
    steps = np.bincount([s for s, *_ in win])
    print(f"frame {args.frame}: {n} keypoints, steps {dict(enumerate(steps.tolist()))}")
    print(f"per-keypoint DMA (k_describe_u2): {per_kp / 1e6:.2f} MB per frame = "
          f"{per_kp / ii_bytes:.2f} x the integral image ({ii_bytes / 1e6:.2f} MB), "
          f"{per_kp / n / 1024:.1f} KiB per keypoint")
    # a wave per keypoint pair: greedy pairs of the same step, nearest in
    # (row, column); the pair DMAs the union of its rows, each row over the
    # union of the two column spans when they overlap (else both spans)
    left = sorted(range(n), key=lambda k: (win[k][0], win[k][2], win[k][1]))
    used, pair_b, npair = set(), 0, 0
    for a in left:
        if a in used:
            continue
        used.add(a)
        sa, xa, ya, ra, ca, wa = win[a]
        best, bsave = None, 0
        for b in left:
            if b in used or win[b][0] != sa or abs(win[b][2] - ya) > 2 * 40 * sa:
                continue
            _, xb, yb, rb, cb, wb = win[b]
            lo, hi = max(ca, cb), min(ca + 4 * wa, cb + 4 * wb)
            save = len(ra & rb) * max(hi - lo, 0) * 4
            if save > bsave:
                best, bsave = b, save
        if best is None:
            pair_b += len(ra) * wa * 16
            continue
        used.add(best)
        npair += 1
        pair_b += len(ra) * wa * 16 + len(win[best][3]) * win[best][5] * 16 - bsave
    print(f"keypoint pairs (same step, best overlap): {npair} pairs, {pair_b / 1e6:.2f} MB per frame "
          f"({pair_b / per_kp:.2f} x per-keypoint)")
    lds = 160 * 1024
    for T in (16, 32, 64, 128):
        tot, fits, tiles = 0, 0, 0
        for ty in range(0, H, T):
            for tx in range(0, W, T):
                sel = [w for w in win if ty <= w[2] < ty + T and tx <= w[1] < tx + T]
                if not sel:
                    continue
                tiles += 1
                r0 = min(min(w[3]) for w in sel)
                r1 = max(max(w[3]) for w in sel) + 1
                c0 = min(w[4] for w in sel)
                c1 = max(w[4] + 4 * w[5] for w in sel)
                b = (r1 - r0) * (c1 - c0) * 4
                tot += b
                fits += b <= lds
        print(f"tile core {T:3d}x{T:<3d}: {tiles:5d} tiles, bounding boxes {tot / 1e6:7.2f} MB per frame "
              f"({tot / per_kp:.2f} x per-keypoint), {fits / tiles:.0%} of tiles fit 160 KiB of LDS")
    return 0


if __name__ == "__main__":
    sys.exit(main())
