#!/usr/bin/env python3
"""Count the work of k_describe_rot's sample walk (config #5) on the CPU.

VERDICT r04 asked how much of the rotated descriptor's per-sample work is
redundant: each of a wave's 50 cell lanes (25 floor cells x 2 row parities)
walks the inverse-rotated box of its cell row by row, over the sj interval
where the cell's two slabs cross the row (widened by kSlack), and rejects
samples that are not its own by the exact membership test -- the model here
restates that loop (surfhip_kernels.hip, k_describe_rot: grid box, row_range,
membership and border tests) in float32 numpy for the keypoints the oracle
finds on synthetic 4K frames, and reports per keypoint:

  * trips    -- iterations of the wave's while loop (max over its lanes: a
                lane that finished idles until the last one does);
  * visited  -- samples the lanes test (sum over lanes);
  * accepted -- samples that pass membership and the border test (each one
                costs the 12 integral gathers and the bin FMAs);
  * gather trips -- trips in which at least one lane accepts (the wave then
                runs the gather path; the other lanes are masked off).

Lane utilisation of the gather path = accepted / (gather trips x 64).
Orientation via np.sin / np.cos instead of the kernel's polynomial: counts
may differ by a sample here and there, not in distribution.

  python3 tools/rot_walk_count.py [--frames 1] [--points 3000]
"""
import argparse
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
f32 = np.float32


def walk(p, W, iH, mag=3, wsz=4, tight=False):
    """One keypoint: (trips, visited, accepted, gather_trips)."""
    NC = wsz + 1
    fw = f32(wsz)
    wofs = f32(wsz * 0.5 - 0.5)
    scale = f32(1.65) * f32(p["scale"])
    step = max(int(np.rint(scale * f32(0.5))), 1)
    x, y = f32(p["x"]), f32(p["y"])
    ix, iy = int(np.rint(x)), int(np.rint(y))
    spacing = scale * f32(mag)
    hs = int(scale)
    rlim, clim = iH - 1 - hs, W - hs
    fracx, fracy = x - f32(ix), y - f32(iy)
    ori = float(p["ori"])
    sine, cose = f32(np.sin(ori)), f32(np.cos(ori))
    fracc = (-sine) * fracy + cose * fracx
    fracr = cose * fracy + sine * fracx
    iradius = int(np.rint(((f32(1.4) * spacing) * f32(wsz + 1)) * f32(0.5) / f32(step)))
    fstep = f32(step)
    seqs = []
    visited = accepted = 0
    for cidx in range(NC * NC):
        cri, cci = cidx // NC - 1, cidx % NC - 1
        A = np.array([((f32(cri + (k >> 1)) - wofs) * spacing + fracr) for k in range(4)], f32)
        B = np.array([((f32(cci + (k & 1)) - wofs) * spacing + fracc) for k in range(4)], f32)
        fi = (cose * A - sine * B) / fstep
        fj = (sine * A + cose * B) / fstep
        if tight:                                    # the box's integer rows / columns only
            i0 = max(-iradius, int(np.ceil(fi.min() - f32(0.05))))
            i1 = min(iradius, int(np.floor(fi.max() + f32(0.05))))
            j0 = max(-iradius, int(np.ceil(fj.min() - f32(0.05))))
            j1 = min(iradius, int(np.floor(fj.max() + f32(0.05))))
        else:
            i0 = max(-iradius, int(np.floor(fi.min())) - 1)
            i1 = min(iradius, int(np.ceil(fi.max())) + 1)
            j0 = max(-iradius, int(np.floor(fj.min())) - 1)
            j1 = min(iradius, int(np.ceil(fj.max())) + 1)
        Alo = ((f32(cri) - wofs) * spacing + fracr) / fstep
        Ahi = ((f32(cri + 1) - wofs) * spacing + fracr) / fstep
        Blo = ((f32(cci) - wofs) * spacing + fracc) / fstep
        Bhi = ((f32(cci + 1) - wofs) * spacing + fracc) / fstep
        use_s, use_c = abs(sine) > 1e-3, abs(cose) > 1e-3
        inv_s = f32(1) / sine if use_s else f32(0)
        inv_c = f32(1) / cose if use_c else f32(0)
        for half in range(2):
            seq = []
            for si in range(i0 + half, i1 + 1, 2):
                fi_ = f32(si)
                lo, hi = f32(j0), f32(j1)
                if use_s:
                    a, b = (Alo - cose * fi_) * inv_s, (Ahi - cose * fi_) * inv_s
                    lo, hi = max(lo, min(a, b) - f32(0.05)), min(hi, max(a, b) + f32(0.05))
                if use_c:
                    a, b = (Blo + sine * fi_) * inv_c, (Bhi + sine * fi_) * inv_c
                    lo, hi = max(lo, min(a, b) - f32(0.05)), min(hi, max(a, b) + f32(0.05))
                if tight:                            # integers inside [lo, hi] only
                    rlo, rhi = max(int(np.ceil(lo)), j0), min(int(np.floor(hi)), j1)
                else:
                    rlo, rhi = max(int(np.floor(lo)), j0), min(int(np.ceil(hi)), j1)
                if rhi >= rlo:
                    cj = np.arange(rlo, rhi + 1)
                    fj_ = cj.astype(f32)
                    rpos = (fstep * (cose * fi_ + sine * fj_) - fracr) / spacing
                    cpos = (fstep * ((-sine) * fi_ + cose * fj_) - fracc) / spacing
                    rx, cx = rpos + wofs, cpos + wofs
                    inb = (rx > -1) & (rx < fw) & (cx > -1) & (cx < fw)
                    ri = np.where(rx >= 0, rx, rx - 1).astype(np.int32)
                    ci = np.where(cx >= 0, cx, cx - 1).astype(np.int32)
                    r, c = iy + si * step, ix + cj * step
                    ok = inb & (ri == cri) & (ci == cci) & (r >= 1 + hs) & (r < rlim) & (c >= 1 + hs) & (c < clim)
                    seq.extend(ok.tolist())
                    visited += len(cj)
                    accepted += int(ok.sum())
                seq.append(False)                    # the trip that moves to the next row
            if i0 + half > i1:
                seq = []
            seqs.append(seq)
    T = max((len(s) for s in seqs), default=0)
    M = np.zeros((len(seqs), T), bool)
    for k, s in enumerate(seqs):
        M[k, :len(s)] = s
    return T, visited, accepted, int(M.any(axis=0).sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1)
    ap.add_argument("--points", type=int, default=3000)
    ap.add_argument("--thresh", type=float, default=4.0)
    ap.add_argument("--tight", action="store_true", help="row intervals rounded inwards")
    a = ap.parse_args()
    surf = importlib.import_module("cuda-surf_amd")
    import oracle as orc
    W, H = 3840, 2160
    p = orc.make_param(5, a.thresh, False, 9, 2, False, True, 4)
    pts = []
    frames = surf.synth_frames(a.frames, W, H)
    for f in range(a.frames):
        got, _, _ = orc.detect(p, frames[f], W, H, max_pts=65536, desc=True)
        pts.append(got)
    pts = np.concatenate(pts)
    rng = np.random.default_rng(0)
    sel = rng.choice(len(pts), size=min(a.points, len(pts)), replace=False)
    res = np.array([walk(pts[i], W, H + 1, tight=a.tight) for i in sel], np.int64)
    trips, vis, acc, gtr = res.T
    n = len(sel)
    print(f"keypoints: {len(pts)} on {a.frames} frame(s), {n} walked")
    print(f"per keypoint: trips {trips.mean():.1f}, visited {vis.mean():.1f}, accepted {acc.mean():.1f}, "
          f"gather trips {gtr.mean():.1f}")
    print(f"accepted / visited {acc.sum() / vis.sum():.3f}; "
          f"lane use of the gather path {acc.sum() / (gtr.sum() * 64):.3f} of 64 lanes "
          f"({acc.sum() / (gtr.sum() * 50):.3f} of the 50 cell lanes); "
          f"gather trips / trips {gtr.sum() / trips.sum():.3f}")
    print(f"ideal gather trips (accepted / 64): {acc.mean() / 64:.1f} per keypoint")


if __name__ == "__main__":
    main()
