"""Host model of k_describe_u2's LDS-DMA ring addressing (surfhip_desc_u2.inc):
for a keypoint, which integral entry each slot word holds after each step's
DMA, and whether every Haar read of a used sample finds the entry it needs.
A checker for the kernel's index math only (no timing).

    python3 tools/u2_ring_check.py x y scale [ring]
"""
import sys

import numpy as np

f32 = np.float32
W, H = 1920, 1080
IW = W + 1
IP = (IW + 127) // 128 * 128
IH = H + 1
MAG, WSZ = 3, 4


def check(x, y, sc, R=6, verbose=True):
    scale = f32(1.65) * f32(sc)
    step = max(int(np.rint(scale * f32(0.5))), 1)
    ix, iy = int(np.rint(f32(x))), int(np.rint(f32(y)))
    dx0, dy0 = f32(x) - f32(ix), f32(y) - f32(iy)
    spacing = scale * f32(MAG)
    hs = int(scale)
    rlim, clim = IH - 1 - hs, W - hs
    iradius = int(np.rint(((spacing * f32(WSZ + 1)) * f32(0.5)) / f32(step)))
    side = 2 * iradius + 1
    fw, wofs = f32(WSZ), f32(WSZ * 0.5 - 0.5)
    lanes = np.arange(64)
    sit = lanes - iradius
    rpos = (f32(1) * (step * sit).astype(f32) - dy0) / spacing
    rx = rpos + wofs
    r_t = iy + sit * step
    rvalid = (lanes < side) & (rx > -1) & (rx < fw) & (r_t >= 1 + hs) & (r_t < rlim)
    vm = np.nonzero(rvalid)[0]
    t0, nv = (int(vm[0]), len(vm)) if len(vm) else (0, 0)
    hmode = hs - 2 * step
    share = hmode in (0, -1)
    cs_ = (ix + (-2 - iradius) * step) & ~3
    W4_ = (ix + (side + 1 - iradius) * step + 2 - cs_ + 3) >> 2
    wide64 = W4_ > 32
    dual = side <= 32 and not (wide64 and W4_ <= 64)
    j = lanes & 31 if dual else lanes
    h = lanes >> 5 if dual else np.zeros(64, int)
    sj = j - iradius
    cpos = ((step * sj).astype(f32) - dx0) / spacing
    cx = cpos + wofs
    c = ix + sj * step
    col_on = (j < side) & (cx > -1) & (cx < fw) & (c >= 1 + hs) & (c < clim)
    G = 2 if dual else 1
    cs = (ix + (-2 - iradius) * step) & ~3
    W4 = (ix + (side + 1 - iradius) * step + 2 - cs + 3) >> 2
    seg = share and W4 <= 64 and (wide64 or step <= 3)
    info = dict(step=step, hs=hs, side=side, dual=dual, W4=W4, seg=seg, t0=t0, nv=nv)
    if not seg:
        return info, []
    RSW = 64 if W4 <= 16 else (128 if W4 <= 32 else 256)
    cpr = RSW // 4
    nd = (2 * G * cpr + 63) // 64
    ip4 = IP * 4
    ck = np.full((2, 64), None, object)
    for i in range(2):
        kk = lanes + 64 * i
        rr, q = kk // cpr, kk % cpr
        for k in range(64):
            if rr[k] < 2 * G and q[k] < W4:
                ck[i, k] = ((iy + (t0 + (rr[k] >> 1) - iradius) * step + (rr[k] & 1)) * IP + cs + 4 * q[k]) * 4
    xo = np.where(j < side, c - cs, 2 * hs)
    b2 = h * 2 * RSW + xo
    errs = []
    for ph in range(1 if dual else 2):
        pb = 0 if dual else ph
        hh = h if dual else np.full(64, ph)
        nstep = np.maximum(nv - hh + 1, 0) >> 1
        nmax = (max(nv + 1, 0) >> 1) if dual else int(nstep[0])
        if nmax == 0:
            continue
        dstep = 2 * step * ip4
        # slot contents: slot -> (step, word -> int index)
        slots = {}

        def dma(s):
            sl = (s + 1) % R
            words = {}
            for i in range(nd):
                for k in range(64):
                    if ck[i, k] is None:
                        continue
                    off = ck[i, k] + (pb - 2) * step * ip4 + (s + 1) * dstep
                    kk = k + 64 * i
                    for e in range(4):
                        words[4 * kk + e] = off // 4 + e
            slots[sl] = (s, words)

        def expect(lane, s):
            t = t0 + int(hh[lane]) + 2 * s
            r = iy + (t - iradius) * step
            cc = int(c[lane])
            return [(r + e) * IP + cc + dc for e in (0, 1) for dc in (-hs, 0, 1, hs + 1)]

        def read(lane, s):
            sl = (s + 1) % R
            st, words = slots.get(sl, (None, {}))
            if st != s:
                return None
            base = int(b2[lane])
            return [words.get(base + e * RSW + dc) for e in (0, 1) for dc in (-hs, 0, 1, hs + 1)]

        for s in range(-1, R - 1):
            dma(s)
        for s in (-1, 0):
            for lane in range(64):
                if col_on[lane] and any(0 <= m < nstep[lane] for m in (s, s + 1)):
                    got, exp = read(lane, s), expect(lane, s)
                    if got != exp:
                        errs.append((ph, "init", s, lane, got, exp))
        n4 = 0
        while n4 < nmax:
            for U in range(R):
                n = n4 + U
                dma(n + R - 1)
                # sample n uses the row sets of steps n - 1, n, n + 1 (read at steps n - 2 .. n)
                # the read of step n + 1's set happens now, from slot (n + 2) % R
                for lane in range(64):
                    if not col_on[lane]:
                        continue
                    s = n + 1
                    used = any(col_on[lane] and m < nstep[lane] for m in (s - 1, s, s + 1) if m >= 0)
                    if not used:
                        continue
                    got = read(lane, s)
                    exp = expect(lane, s)
                    if got != exp:
                        errs.append((ph, n, lane, got, exp))
            n4 += R
    if verbose:
        print(info, "errors", len(errs), errs[:3])
    return info, errs


if __name__ == "__main__":
    a = sys.argv[1:]
    R = int(a[3]) if len(a) > 3 else 6
    check(float(a[0]), float(a[1]), float(a[2]), R)
