"""CPU tests of the oracle (no GPU): known-answer tests against closed forms
and an independent numpy restatement, geometry against the values SURVEY.md
derives from the reference's host code, and the frozen golden vectors."""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, REF_DATA, assert_points_equal, desc_l2

F32 = np.float32


def test_struct_layouts(orc):
    import ctypes as C
    assert C.sizeof(orc.Param) == 48
    assert orc.POINT_DTYPE.itemsize == 48
    # offsets of surf_structures.h:10-30 / 45-72
    assert orc.Param.doubled.offset == 8 and orc.Param.upright.offset == 28
    assert orc.Param.extend.offset == 29 and orc.Param.nfeatures.offset == 44
    assert [orc.POINT_DTYPE.fields[k][1] for k in ("o", "laplace", "ori", "ambiguity")] == [12, 20, 24, 44]


def test_init_params_match_reference_defaults(orc):
    """Surfor::init (surf.cpp:60-79) with main.cpp's arguments."""
    p = orc.make_param(4, 4.0, False, 9, 2, True, False, 4)
    assert (p.init_lobe, p.max_scale, p.sampling, p.mag_factor, p.orient_size, p.nfeatures) == (3, 5, 2, 3, 4, 64)
    assert p.divisor == 1.0
    p = orc.make_param(5, 4.0, False, 9, 2, False, True, 4)
    assert (p.orient_size, p.nfeatures) == (8, 128)
    p = orc.make_param(4, 4.0, True, 9, 2)     # doubled (surf.cpp:69, 72)
    assert (p.sampling, p.divisor, p.doubled) == (4, 0.5, True)


def test_geometry_1080p_matches_survey(orc):
    """SURVEY.md 8 notation + Appendix A3 (values computed from surf.cpp:374-392,
    surfd.cu:2846-2864, 3062-3076)."""
    p = orc.make_param(4, 4.0, upright=True)
    g, octs = orc.geometry(p, 1920, 1080)
    assert (g.iwhp.x, g.iwhp.y, g.iwhp.z) == (1921, 1081, 2048)
    assert [(g.swhp[o].x, g.swhp[o].y, g.swhp[o].z) for o in range(4)] == \
        [(960, 540, 1024), (480, 270, 512), (240, 135, 256), (120, 67, 128)]
    assert g.tot_osize == 3_671_680
    o0 = octs[0]
    assert list(o0.mask[:5]) == [3, 5, 7, 9, 11]
    assert list(o0.border1[:5]) == [6, 6, 6, 7, 9]
    assert list(o0.borders[:5]) == [6, 6, 6, 6, 7]
    assert list(o0.mborders)[:2] == [7, 8]
    for o, masks in ((1, [15, 19, 23]), (2, [31, 39, 47]), (3, [63, 79, 95])):
        assert list(octs[o].mask[:3]) == masks
        assert list(octs[o].border1[:3]) == [8, 8, 9]
        assert list(octs[o].borders[:5]) == [8, 8, 8, 8, 8]
        assert list(octs[o].mborders)[:2] == [9, 9]
    # NMS launch extents (grids (30,17,2), (15,8,2), (7,4,2), (4,2,2) of 16x16)
    assert [(octs[o].nms_gx // 16, octs[o].nms_gy // 16) for o in range(4)] == [(30, 17), (15, 8), (7, 4), (4, 2)]


def test_hessian_bytes_survey_number(orc):
    """Compulsory Hessian bytes at 1080p = 20,058,324."""
    p = orc.make_param(4, 4.0, upright=True)
    g, octs = orc.geometry(p, 1920, 1080)
    valid = 0
    for o in range(4):
        q = octs[o]
        for i in range(q.nscale):
            b = q.border1[i]
            valid += (g.swhp[o].x - 2 * b) * (g.swhp[o].y - 2 * b)
    assert valid == 2_937_980
    assert 1921 * 1081 * 4 + 4 * valid == 20_058_324


def test_integral_vs_numpy(orc):
    rng = np.random.default_rng(1)
    for w, h in ((1, 1), (7, 3), (64, 48), (333, 101)):
        img = rng.integers(0, 256, (h, w), dtype=np.uint8)
        ii = orc.integral(img, w, h)
        ref = np.zeros((h + 1, w + 1), np.int64)
        ref[1:, 1:] = img.astype(np.int64).cumsum(0).cumsum(1)
        np.testing.assert_array_equal(ii[:, :w + 1], ref)


def test_box_sum_convention(orc):
    """getSum(x1, y1, x2, y2) sums the inclusive rect [x2..x1] x [y2..y1]
    (surfd.cu:334-343)."""
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (40, 50), dtype=np.uint8)
    ii = orc.integral(img, 50, 40)
    for _ in range(50):
        x2, y2 = rng.integers(0, 45), rng.integers(0, 35)
        x1, y1 = x2 + rng.integers(0, 4), y2 + rng.integers(0, 4)
        got = orc.lib.or_test_box(ii.ctypes.data, ii.shape[1], int(x1), int(y1), int(x2), int(y2))
        assert got == img[y2:y1 + 1, x2:x1 + 1].astype(np.int64).sum()


def _np_hessian(img, w, h, p, g, octs):
    """Independent numpy float32 restatement of getHessian * norm (surfd.cu:353-366,
    445-481) for octave 0, computed from box sums of the image itself."""
    ii = np.zeros((h + 1, w + 1), np.int64)
    ii[1:, 1:] = img[:, :w].astype(np.int64).cumsum(0).cumsum(1)

    def S(x1, y1, x2, y2):
        return ii[y1 + 1, x1 + 1] + ii[y2, x2] - ii[y2, x1 + 1] - ii[y1 + 1, x2]

    q = octs[0]
    out = {}
    for i in range(q.nscale):
        m, x2, x3, x4 = q.mask[i], q.x2[i], q.x3[i], q.x4[i]
        b = q.border1[i]
        sw, sh = g.swhp[0].x, g.swhp[0].y
        plane = np.zeros((sh, sw), F32)
        iy, ix = np.mgrid[b:sh - b, b:sw - b]
        X, Y = q.delta * ix, q.delta * iy
        dxx = (S(X + m + x2, Y + x3, X - m - x2, Y - x3) - 3 * S(X + x2, Y + x3, X - x2, Y - x3)).astype(F32)
        dyy = (S(X + x3, Y + m + x2, X - x3, Y - m - x2) - 3 * S(X + x3, Y + x2, X - x3, Y - x2)).astype(F32)
        dxy = F32(0.6) * (S(X + x4, Y, X, Y - x4) + S(X, Y + x4, X - x4, Y) - S(X + x4, Y + x4, X, Y)
                          - S(X, Y, X - x4, Y - x4)).astype(F32)
        r = F32(0.003921568627)
        plane[b:sh - b, b:sw - b] = (r * r) * (dxx * dyy - dxy * dxy) * F32(q.norm[i])
        out[i] = plane
    return out


def test_hessian_octave0_vs_numpy(orc, surf):
    w, h = 200, 150
    img = surf.synth_frames(1, w, h, first=5)[0]
    p = orc.make_param(4, 4.0, upright=True)
    ii, resp, g, octs = orc.hessian(p, img, w, h)
    ref = _np_hessian(img, w, h, p, g, octs)
    sw, sh, sp = g.swhp[0].x, g.swhp[0].y, g.swhp[0].z
    for i, plane in ref.items():
        got = resp[i * g.osize[0]: (i + 1) * g.osize[0]].reshape(sh, sp)[:, :sw]
        np.testing.assert_array_equal(got.view(np.uint32), plane.view(np.uint32))


def test_halfimage_planes(orc, surf):
    """Planes 0/1 of octave o > 0 are planes 2/4 of octave o-1 at (2r, 2c)
    (halfImage, surfd.cu:321-331; surf.cpp:252-258)."""
    w, h = 320, 240
    img = surf.synth_frames(1, w, h, first=9)[0]
    p = orc.make_param(4, 4.0, upright=True)
    _, resp, g, _ = orc.hessian(p, img, w, h)
    for o in range(1, 4):
        sw, sh, sp = g.swhp[o].x, g.swhp[o].y, g.swhp[o].z
        psw, psh, psp = g.swhp[o - 1].x, g.swhp[o - 1].y, g.swhp[o - 1].z
        for dst, src in ((0, 2), (1, 4)):
            d = resp[g.ooff[o] + dst * g.osize[o]:][:sh * sp].reshape(sh, sp)[:, :sw]
            s = resp[g.ooff[o - 1] + src * g.osize[o - 1]:][:psh * psp].reshape(psh, psp)
            np.testing.assert_array_equal(d, s[0:2 * sh:2, 0:2 * sw:2])


def test_solver_closed_form(orc):
    """solveLinearSystem (surfd.cu:835-887) on well-conditioned systems."""
    rng = np.random.default_rng(3)
    for _ in range(20):
        A = rng.normal(size=(3, 3)).astype(F32) + 3 * np.eye(3, dtype=F32)
        x = rng.normal(size=3).astype(F32)
        b = (A.astype(np.float64) @ x.astype(np.float64)).astype(F32)
        sol = b.copy()
        sq = A.copy().ravel()
        orc.lib.or_test_solve3(sol.ctypes.data, sq.ctypes.data)
        np.testing.assert_allclose(sol, x, rtol=1e-4, atol=1e-4)


def test_place_in_index_weights_sum_to_mag(orc):
    """placeInIndex (surfd.cu:1199-1271): for interior (rx, cx) the bilinear
    weights put exactly mag1 + mag2 into the descriptor."""
    rng = np.random.default_rng(4)
    for _ in range(200):
        d = np.zeros(64, F32)
        rx, cx = rng.uniform(0, 3, 2).astype(F32)
        m1, m2 = rng.uniform(-1, 1, 2).astype(F32)
        orc.lib.or_test_place(d.ctypes.data, 4, 4, float(m1), 0, float(m2), 2, float(rx), float(cx))
        assert abs(d.sum() - (m1 + m2)) < 1e-5
        assert abs(d[0::4].sum() - m1) < 1e-5 and abs(d[2::4].sum() - m2) < 1e-5


def test_luts(orc):
    l1, l2, b = orc.tables()
    n = np.arange(83)
    np.testing.assert_allclose(l1, np.exp(-(n + 0.5) / 12.5), rtol=1e-6)
    np.testing.assert_allclose(l2, np.exp(-(np.arange(40) + 0.5) / 8), rtol=1e-6)
    assert b[0] == F32(-np.pi)
    np.testing.assert_allclose(np.diff(b), 2 * np.pi / 72, rtol=1e-4)


def test_sincos_and_atan2(orc):
    for x in np.linspace(-4.5, 4.5, 2001, dtype=F32):
        assert abs(orc.lib.or_sinf(float(x)) - np.sin(np.float64(x))) < 3e-7
        assert abs(orc.lib.or_cosf(float(x)) - np.cos(np.float64(x))) < 3e-7
    rng = np.random.default_rng(5)
    for y, x in rng.normal(size=(2000, 2)).astype(F32):
        assert abs(orc.lib.or_fast_atan2(float(y), float(x)) - np.arctan2(y, x)) < 3e-4   # 3-term polynomial


def test_blob_detected_at_center(orc):
    """A single dark-on-bright Gaussian blob yields a keypoint at its centre."""
    w, h = 256, 256
    yy, xx = np.mgrid[0:h, 0:w]
    sigma, cx, cy = 6.0, 128.3, 121.7
    img = np.clip(200 - 150 * np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * sigma ** 2)), 0, 255)
    img = np.round(img).astype(np.uint8)
    p = orc.make_param(4, 4.0, upright=True)
    pts, desc, _ = orc.detect(p, img, w, h)
    assert len(pts) >= 1
    k = np.argmax(pts["strength"])
    assert abs(pts["x"][k] - cx) < 1.0 and abs(pts["y"][k] - cy) < 1.0
    # scale ~ 1.2/9 of the box size; a blob of sigma s peaks near lobe ~ s*2.5
    assert 3.0 < pts["scale"][k] < 12.0
    assert pts["laplace"][k] == 1                   # dark blob on bright background: positive trace
    np.testing.assert_allclose(np.linalg.norm(desc[k]), 1.0, rtol=1e-5)


def test_upright_descriptor_flip_symmetry(orc):
    """Mirroring the image left-right mirrors the upright descriptor cells and
    flips the sign of the dx bins (an independent property check)."""
    w, h = 160, 160
    rng = np.random.default_rng(6)
    img = np.clip(rng.normal(128, 40, (h, w)), 0, 255).astype(np.uint8)
    yy, xx = np.mgrid[0:h, 0:w]
    img = np.clip(img * 0.2 + 200 - 150 * np.exp(-((xx - 80) ** 2 + (yy - 80) ** 2) / 50.0), 0, 255).astype(np.uint8)
    p = orc.make_param(4, 4.0, upright=True)
    pts, desc, _ = orc.detect(p, img, w, h)
    assert len(pts) > 0
    assert np.allclose(np.linalg.norm(desc, axis=1), 1.0, atol=1e-5)


# -------------------------------------------------------------- goldens

GOLDEN_CASES = ["left_1280x960_upright", "left_1280x960_rotated", "right_1280x960_upright",
                "left_640x480_upright", "left_1280x960_rotated_ext"]


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_oracle_matches_golden(orc, name):
    """The oracle reproduces the frozen vectors (tests/golden, generated by
    tests/golden/make_golden.py from the reference's data/*.pgm)."""
    path = os.path.join(GOLDEN, name + ".npz")
    if not os.path.exists(path):
        pytest.skip("golden fixtures not generated")
    z = np.load(path)
    img = np.load(os.path.join(GOLDEN, "images.npz"))[str(z["image_key"])]
    h, w = img.shape
    upright, extend = bool(z["meta"][0]), bool(z["meta"][1])
    p = orc.make_param(4, 4.0, False, 9, 2, upright, extend, 4)
    pts, desc, nc = orc.detect(p, img, w, h)
    ref = np.frombuffer(z["points"].tobytes(), dtype=orc.POINT_DTYPE)
    assert_points_equal(pts, ref, fields=("x", "y", "scale", "o", "strength", "laplace", "ori"))
    assert desc_l2(desc, z["desc"]).max() == 0.0
    assert nc == int(z["meta"][2])


# ------------------------------------------------------------------ match
def _np_match(f1, f2, full_tail=False):
    """Independent restatement of findMaxCorr (surfd.cu:2530-2656) for inputs
    whose dot products are exact in fp32 (dyadic values): every score is the
    exact integer-scaled sum, so the FMA chain order cannot matter.  Thread
    row g of the reference block sees the p2 with (p2 % 32) // 4 == g of the
    full tiles (surfd.cu:2569), top-2 by strict '>' from (0, 0, -1), rows
    merged in order ignoring their second scores (surfd.cu:2638-2655)."""
    n1, n2 = len(f1), len(f2)
    nscan = n2 if full_tail else 32 * (n2 // 32)
    scores = (f1.astype(np.float64) @ f2.astype(np.float64).T)[:, :nscan]
    rows = (np.arange(nscan) % 32) // 4
    out = []
    for p1 in range(n1):
        states = []
        for g in range(8):
            idx = np.nonzero(rows == g)[0]
            mx, sc, ix = 0.0, 0.0, -1
            for p2 in idx:
                s = scores[p1, p2]
                if s > mx:
                    sc, mx, ix = mx, s, int(p2)
                elif s > sc:
                    sc = s
            states.append((mx, sc, ix))
        M, S, I = states[0]
        for mx, _sc, ix in states[1:]:
            if ix == I:
                continue
            if mx > M:
                S, M, I = max(M, S), mx, ix
            elif mx > S:
                S = mx
        out.append((M, S, I))
    return out


@pytest.mark.parametrize("n1,n2,nf,full", [(37, 100, 64, False), (37, 100, 64, True), (5, 31, 64, False),
                                            (5, 31, 64, True), (64, 96, 128, False), (20, 70, 36, True)])
def test_match_vs_numpy_exact(orc, n1, n2, nf, full):
    rng = np.random.default_rng(n1 * 1000 + n2 + nf + full)
    # multiples of 1/8 in [-1, 1]: products are multiples of 1/64, sums stay
    # far below 2^24 / 64, so every fp32 FMA chain is exact
    f1 = (rng.integers(-8, 9, (n1, nf)) / 8).astype(np.float32)
    f2 = (rng.integers(-8, 9, (n2, nf)) / 8).astype(np.float32)
    f2[7] = f1[3]                                      # exact duplicate -> ties within rows
    f2[min(40, n2 - 1)] = f1[3]
    p1 = np.zeros(n1, orc.POINT_DTYPE)
    p2 = np.zeros(n2, orc.POINT_DTYPE)
    p2["x"] = np.arange(n2) + 0.5
    p2["y"] = -np.arange(n2) - 0.25
    got = orc.match(p1, p2, f1, f2, full_tail=full)
    ref = _np_match(f1, f2, full)
    for i, (M, S, I) in enumerate(ref):
        assert got["match"][i] == I, i
        assert got["score"][i] == np.float32(M), i
        assert got["ambiguity"][i] == np.float32(np.float32(S) / (np.float32(M) + np.float32(1e-6))), i
        assert got["match_x"][i] == (p2["x"][I] if I >= 0 else 0.0)
        assert got["match_y"][i] == (p2["y"][I] if I >= 0 else 0.0)
    if n2 < 32 and not full:                           # no full tile: nothing is scored
        assert (got["match"] == -1).all()


def test_match_tail_bug_is_the_default(orc):
    """The reference never scores the last partial tile of set 2
    (surfd.cu:2569): a perfect partner there is not found by default."""
    rng = np.random.default_rng(3)
    f = rng.standard_normal((40, 64)).astype(np.float32)
    f /= np.linalg.norm(f, axis=1, keepdims=True)
    p = np.zeros(40, orc.POINT_DTYPE)
    q = orc.match(p[35:36], p, f[35:36], f)
    assert q["match"][0] != 35
    q = orc.match(p[35:36], p, f[35:36], f, full_tail=True)
    assert q["match"][0] == 35


def test_match_golden_fixture(orc):
    z = np.load(os.path.join(GOLDEN, "match_left_right_upright.npz"))
    a = np.load(os.path.join(GOLDEN, "left_1280x960_upright.npz"))
    b = np.load(os.path.join(GOLDEN, "right_1280x960_upright.npz"))
    p1, p2 = a["points"].view(orc.POINT_DTYPE), b["points"].view(orc.POINT_DTYPE)
    for tag, full in (("ref", False), ("full", True)):
        m = orc.match(p1, p2, a["desc"], b["desc"], full_tail=full)
        for f in ("score", "match", "match_x", "match_y", "ambiguity"):
            np.testing.assert_array_equal(m[f].view(np.uint32) if m[f].dtype == np.float32 else m[f],
                                          z[f"{tag}_{f}"].view(np.uint32) if z[f"{tag}_{f}"].dtype == np.float32
                                          else z[f"{tag}_{f}"])
    # left/right overlap with a ~(532, -18) px shift: the unambiguous matches
    # (ambiguity < 0.9) agree on that displacement
    s = z["ref_ambiguity"] < 0.9
    dx = p1["x"][s] - z["ref_match_x"][s]
    dy = p1["y"][s] - z["ref_match_y"][s]
    assert s.sum() > 100
    assert ((abs(dx - np.median(dx)) < 40) & (abs(dy - np.median(dy)) < 40)).mean() > 0.95


# ---------------------------------------------------------- doubled image
def _sim_reference_double_integral(img):
    """Literal simulation of cuIntegralDoubleU4's six kernels
    (surfd.cu:166-318, launch geometry surfd.cu:2707-2772) on a zeroed
    buffer with spare rows, every thread of every launch run in turn (no
    thread reads what another thread of the same launch writes)."""
    h1, w1 = img.shape
    src = np.zeros((h1 + 1, w1 + 2), np.int64)          # the reads past the image see 0
    src[:h1, :w1] = img
    w2, h2 = 2 * w1 - 1, 2 * h1 - 1
    p2 = (w2 + 127) // 128 * 128
    dst = np.zeros(((h2 + 3) * p2,), np.int64)         # spare rows take the OOB writes

    def rn(v):
        return int(np.rint(np.float32(v)))
    # integralDoubleRow0U2: thread (ix, iy), bix = 2 ix
    for iy in range(h1):
        for bix in range(0, w1, 2):
            S = lambda y, x: int(src[y, x])
            w_ = (2 * iy + 1) * p2 + 2 * bix + 1
            x_, y_, z_ = w_ + 1, w_ + p2, w_ + p2 + 1
            s00, s01, s10, s11 = S(iy, bix), S(iy, bix + 1), S(iy + 1, bix), S(iy + 1, bix + 1)
            dst[w_] = s00
            dst[y_] = rn(np.float32(s00 + s10) * np.float32(0.5))
            if bix + 1 >= w1:
                continue
            dst[x_] = dst[w_] + rn(np.float32(s00 + s01) * np.float32(0.5))
            dst[z_] = dst[y_] + rn(np.float32(s00 + s01 + s10 + s11) * np.float32(0.25))
            s00, s01, s10, s11 = s01, S(iy, bix + 2), s11, S(iy + 1, bix + 2)
            w_, x_, y_, z_ = w_ + 2, x_ + 2, y_ + 2, z_ + 2
            dst[w_] = dst[w_ - 1] + s00
            dst[y_] = dst[y_ - 1] + rn(np.float32(s00 + s10) * np.float32(0.5))
            if bix + 2 >= w1:
                continue
            dst[x_] = dst[w_] + rn(np.float32(s00 + s01) * np.float32(0.5))
            dst[z_] = dst[y_] + rn(np.float32(s00 + s01 + s10 + s11) * np.float32(0.25))
    # integralRow1U4: per row iy >= 1, chain the ends of the 4-column groups
    for iy in range(1, h2):
        i = iy * p2 + 1 + 3
        j, k = i + 4, 8
        while k < w2:
            dst[j] += dst[i]
            i, j, k = j, j + 4, k + 4
    # integralRow2U4: add the previous group's end to columns 4(ix+1)+1 .. +3
    for iy in range(1, h2):
        for ix in range(0, (w2 - 1) // 4 + 1):
            bix = (ix + 1) * 4 + 1
            if bix >= w2:
                continue
            idx = iy * p2 + bix - 1
            for t in range(3):
                if bix + t >= w2:
                    break
                dst[idx + 1 + t] += dst[idx]
    # integralCol0U4: within groups of 4 rows starting at row 1
    for ix in range(1, w2):
        for iy in range(0, (h2 - 1) // 4 + 1):
            biy = iy * 4 + 1
            if biy + 1 >= h2:
                continue
            idx = biy * p2 + ix
            for t in range(3):
                if biy + 1 + t >= h2:
                    break
                dst[idx + p2] += dst[idx]
                idx += p2
    # integralCol1U4: chain the group ends (rows 4, 8, ...)
    for ix in range(1, w2):
        i = ix + 4 * p2
        j, k = i + 4 * p2, 8
        while k < h2:
            dst[j] += dst[i]
            i, j, k = j, j + 4 * p2, k + 4
    # integralCol2U4: add the previous group's end to rows 4(iy+1)+1 .. +3
    for ix in range(1, w2):
        for iy in range(0, (h2 - 1) // 4 + 1):
            biy = (iy + 1) * 4 + 1
            if biy >= h2:
                continue
            idx = (biy - 1) * p2 + ix
            for t in range(3):
                if biy + t >= h2:
                    break
                dst[idx + (1 + t) * p2] += dst[idx]
    return dst[:h2 * p2].reshape(h2, p2)[:, :w2].astype(np.uint32).view(np.int32)


@pytest.mark.parametrize("h,w", [(7, 9), (6, 10), (9, 12), (5, 5)])
def test_doubled_integral_vs_reference_kernels(orc, h, w):
    """or_double_image + or_integral equals a literal run of the reference's
    six doubled-integral kernels on the (2w-1) x (2h-1) grid."""
    rng = np.random.default_rng(h * 100 + w)
    img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    img[0, 0], img[-1, -1] = 255, 1                   # odd sums: exercise round-half-even
    ref = _sim_reference_double_integral(img)
    D = orc.double_image(img, w, h)
    got = orc.integral(D, 2 * w - 2, 2 * h - 2)[:, :2 * w - 1]
    np.testing.assert_array_equal(got, ref)


def test_doubled_detect_geometry(orc):
    p = orc.make_param(4, 4.0, doubled=True, upright=True)
    assert p.sampling == 4 and p.divisor == np.float32(0.5)
    g, _ = orc.geometry(p, 640, 480)
    assert (g.iwhp.x, g.iwhp.y, g.iwhp.z) == (1279, 959, 1280)      # surf.cpp:377-379
    assert (g.swhp[0].x, g.swhp[0].y) == (319, 239)
    img = np.load(os.path.join(GOLDEN, "images.npz"))["left_640x480"]
    pts, d, nc = orc.detect(p, img, 640, 480)
    assert len(pts) > 500 and nc == len(pts)
    assert pts["x"].max() < 640 and pts["y"].max() < 480       # coordinates in source pixels


@pytest.mark.parametrize("upright,extend", [(True, False), (False, False), (True, True), (False, True)])
def test_doubled_describes_at_twice_the_position(orc, upright, extend):
    """A doubled detector describes a point (x, y, scale) -- source-pixel
    coordinates, makePoint's divisor 0.5 -- in the integral of the 2x frame D
    at (2x, 2y) with 3.3 * scale, and orients it with 2 * scale
    (surfd.cu:1581-1592, 1734-1745, 2406-2417).  Since 3.3f == 2 * 1.65f
    exactly, that is bit for bit the ordinary (not doubled) description of
    the point (2x, 2y, 2 * scale) on D itself; describing (x, y, scale) on D
    (what round 1 did) gives different descriptors."""
    img = np.load(os.path.join(GOLDEN, "images.npz"))["left_640x480"][100:260, 120:360]
    h, w = img.shape
    pd = orc.make_param(4, 4.0, doubled=True, upright=upright, extend=extend)
    pts, desc, _ = orc.detect(pd, img, w, h)
    assert len(pts) > 20
    D = orc.double_image(img, w, h)
    pn = orc.make_param(4, 4.0, doubled=False, upright=upright, extend=extend)
    g, _ = orc.geometry(pn, 2 * w - 2, 2 * h - 2)
    ii = orc.integral(D, 2 * w - 2, 2 * h - 2)
    q = pts.copy()
    q["x"] = pts["x"] * np.float32(2)
    q["y"] = pts["y"] * np.float32(2)
    q["scale"] = pts["scale"] * np.float32(2)
    ori, d2 = orc.describe_points(pn, g, ii, q)
    if not upright:
        np.testing.assert_array_equal(ori.view(np.uint32), pts["ori"].view(np.uint32))
    np.testing.assert_array_equal(d2.view(np.uint32), desc.view(np.uint32))
    _, d_old = orc.describe_points(pn, g, ii, pts, orient=upright)
    assert np.abs(d_old - desc).max() > 0.05


# ---------------------------------------------------------------- pinning
# oracle/_ref/libref_host.so is built by oracle/ref_extract.py from the
# reference's own host C++ (surfd.cu:3082-3186 hSolveLinearSystem and
# hFitQuadrat, surfd.cu:2833-2866 the Hessian parameter recurrence), compiled
# as it stands with g++ -ffp-contract=off.  These tests pin the oracle's
# restatements to it bit for bit.

def _ref_or_skip(orc):
    L = orc.ref_host()
    if L is None:
        if os.path.exists("/root/reference/surfd.cu"):
            import subprocess
            subprocess.check_call([sys.executable, os.path.join(os.path.dirname(orc.__file__), "ref_extract.py")])
            L = orc.ref_host()
        if L is None:
            pytest.skip("reference sources absent: oracle/_ref not built")
    return L


def _solve_cases(n, rng):
    """Random, integer, near-singular, singular, tiny/huge and NaN/inf systems."""
    out = []
    for k in range(n):
        kind = k % 8
        if kind == 0:
            m = rng.standard_normal(9)
        elif kind == 1:
            m = rng.integers(-4, 5, 9).astype(np.float64)
        elif kind == 2:
            m = rng.standard_normal(9)
            m[3:6] = m[0:3] * np.float32(1 + 1e-6)          # nearly dependent rows
        elif kind == 3:
            m = rng.standard_normal(9)
            m[rng.integers(0, 3) * 3 + np.arange(3)] = 0     # a zero row
        elif kind == 4:
            m = rng.standard_normal(9) * 10.0 ** rng.integers(-30, 30, 9)
        elif kind == 5:
            m = rng.standard_normal(9)
            m[[0, 4, 8]] = 0                                  # zero diagonal: forces pivoting
        elif kind == 6:
            m = np.zeros(9)                                   # all zero: 0/0
        else:
            m = rng.standard_normal(9)
            m[rng.integers(0, 9)] = [np.nan, np.inf, -np.inf][k % 3]
        sol = rng.standard_normal(3) * 10.0 ** rng.integers(-3, 4)
        out.append((m.astype(np.float32), sol.astype(np.float32)))
    return out


def test_oracle_solver_pinned_to_reference_host_code(orc):
    L = _ref_or_skip(orc)
    rng = np.random.default_rng(2024)
    cases = _solve_cases(100_000, rng)
    bad = 0
    for m, sol in cases:
        m1, s1 = m.copy(), sol.copy()
        m2, s2 = m.copy(), sol.copy()
        orc.lib.or_test_solve3(s1.ctypes.data, m1.ctypes.data)
        L.ref_solve(s2.ctypes.data, m2.ctypes.data)
        if s1.tobytes() != s2.tobytes() or m1.tobytes() != m2.tobytes():
            bad += 1
    assert bad == 0, f"{bad} of {len(cases)} systems differ from hSolveLinearSystem"


def test_oracle_fit_pinned_to_reference_host_code(orc):
    L = _ref_or_skip(orc)
    rng = np.random.default_rng(7)
    sh, sp = 9, 16
    osize = sh * sp
    n = 0
    for trial in range(4000):
        kind = trial % 4
        planes = rng.standard_normal((3, sh, sp)).astype(np.float32)
        if kind == 1:
            planes *= np.float32(1e4)
        elif kind == 2:                                  # a flat, quantised response field
            planes = np.round(planes * 4).astype(np.float32) / np.float32(4)
        elif kind == 3:
            planes[1, 4, 4] += np.float32(50)            # a clear peak
        src = np.ascontiguousarray(planes.reshape(-1))
        for r, c in ((4, 4), (1, 1), (7, 14), (3, 8)):
            o1 = np.zeros(3, np.float32)
            o2 = np.zeros(3, np.float32)
            v1 = orc.lib.or_test_fit(src.ctypes.data, o1.ctypes.data, 1, r, c, osize, sp)
            v2 = L.ref_fit(src.ctypes.data, o2.ctypes.data, 1, r, c, osize, sp)
            assert np.float32(v1).tobytes() == np.float32(v2).tobytes() or (np.isnan(v1) and np.isnan(v2))
            assert o1.tobytes() == o2.tobytes() or (np.isnan(o1).any() and np.isnan(o2).any())
            n += 1
    assert n == 16000


@pytest.mark.parametrize("noct,sampling,init_mask,doubled", [(4, 2, 9, False), (5, 2, 9, False), (6, 2, 9, False),
                                                              (4, 2, 9, True), (4, 3, 9, False), (4, 1, 9, False)])
def test_oracle_octave_params_pinned_to_reference_host_code(orc, noct, sampling, init_mask, doubled):
    """or_octave_params against surfd.cu:2833-2866 driven the way
    Surfor::detectAndCompute drives it (surf.cpp:240-292: init mask
    init_lobe - 2, border1 per octave, octave doubling)."""
    L = _ref_or_skip(orc)
    p = orc.make_param(noct, 4.0, doubled, init_mask, sampling, True, False, 4)
    g, octs = orc.geometry(p, 1920, 1080)
    ms, mo = 8, 8
    mask_size = C.c_int(p.init_lobe - 2)                 # surf.cpp:240
    octave = 1
    borders = np.zeros(ms, np.int32)
    for o in range(noct):
        if o > 0:                                        # surf.cpp:261-264
            border1 = ((3 * (mask_size.value + 4 * octave)) // 2) // (p.sampling * octave) + 1
            borders[0] = borders[1] = border1
            init_scale = 2
        else:                                            # surf.cpp:269
            border1 = ((3 * (mask_size.value + 6 * octave)) // 2) // (p.sampling * octave) + 1
            init_scale = 0
        params = np.zeros(7 * ms, np.int32)
        norms = np.zeros(ms, np.float32)
        L.ref_hessian_params(g.swhp[o].x, g.swhp[o].y, init_scale, p.max_scale, C.byref(mask_size), border1,
                             borders.ctypes.data, octave, p.sampling, params.ctypes.data, norms.ctypes.data)
        q = octs[o]
        nsc = p.max_scale - init_scale
        assert q.init_scale == init_scale and q.nscale == nsc
        for i in range(nsc):
            assert q.mask[i] == params[i], (o, i)
            assert q.border1[i] == params[ms + i], (o, i)
            assert q.delta == params[3 * ms + i]
            assert (q.x2[i], q.x3[i], q.x4[i]) == (params[4 * ms + i], params[5 * ms + i], params[6 * ms + i])
            assert np.float32(q.norm[i]).tobytes() == norms[i].tobytes()
        assert list(q.borders)[:p.max_scale] == borders[:p.max_scale].tolist(), o
        assert mask_size.value == q.mask[nsc - 1]
        octave += octave


def test_oracle_luts_pinned_to_reference_init_lut(orc):
    """or_init_tables' lookup1 / lookup2 against initLut's own loops
    (surf.cpp:358-371, host expf) bit for bit; the GPU detector uploads the
    same host values (surfhip_api.hip)."""
    L = _ref_or_skip(orc)
    t1 = np.zeros(83, np.float32)
    t2 = np.zeros(40, np.float32)
    L.ref_init_lut(t1.ctypes.data, t2.ctypes.data)
    l1 = np.zeros(83, np.float32)
    l2 = np.zeros(40, np.float32)
    b = np.zeros(72, np.float32)
    orc.lib.or_init_tables(l1.ctypes.data, l2.ctypes.data, b.ctypes.data)
    assert l1.tobytes() == t1.tobytes() and l2.tobytes() == t2.tobytes()


@pytest.mark.parametrize("init_mask", [6, 9, 12, 15, 18, 20])
@pytest.mark.parametrize("sampling,doubled,noct", [(2, False, 4), (2, True, 5), (1, False, 6), (3, False, 4)])
def test_oracle_octave_plan_pinned_to_reference_loop(orc, init_mask, sampling, doubled, noct):
    """Every octave's borders (the NMS's d_borders) and Hessian parameters
    from the reference's own statements (surf.cpp:240 / 261 / 269 in
    surf.cpp:241-293's loop around surfd.cu:2833-2866) against
    or_octave_params, for every initial lobe the reference accepts."""
    L = _ref_or_skip(orc)
    p = orc.make_param(noct, 4.0, doubled, init_mask, sampling, True, False, 4)
    g, octs = orc.geometry(p, 1920, 1080)
    ms = 8
    swx = np.array([g.swhp[o].x for o in range(noct)], np.int32)
    swy = np.array([g.swhp[o].y for o in range(noct)], np.int32)
    borders = np.zeros((noct, 8), np.int32)
    params = np.zeros((noct, 7 * ms), np.int32)
    norms = np.zeros((noct, ms), np.float32)
    L.ref_octave_plan(p.init_lobe, p.sampling, noct, p.max_scale, swx.ctypes.data, swy.ctypes.data,
                      borders.ctypes.data, params.ctypes.data, norms.ctypes.data)
    for o in range(noct):
        q = octs[o]
        nsc = q.nscale
        assert nsc == p.max_scale - (0 if o == 0 else 2)
        assert list(q.mask)[:nsc] == params[o, :nsc].tolist(), o
        assert list(q.border1)[:nsc] == params[o, ms:ms + nsc].tolist(), o
        assert list(q.x2)[:nsc] == params[o, 4 * ms:4 * ms + nsc].tolist()
        assert list(q.x3)[:nsc] == params[o, 5 * ms:5 * ms + nsc].tolist()
        assert list(q.x4)[:nsc] == params[o, 6 * ms:6 * ms + nsc].tolist()
        assert np.array(list(q.norm)[:nsc], np.float32).tobytes() == norms[o, :nsc].tobytes()
        assert list(q.borders)[:p.max_scale] == borders[o, :p.max_scale].tolist(), o
        # the NMS start offsets (surfd.cu:3062-3068) from the same borders
        lev = [k for k in range(1, p.max_scale - 1, 2)]
        assert list(q.mborders)[:len(lev)] == [int(borders[o, k + 1]) + 1 for k in lev]


def test_oracle_sanitizer_build():
    """ASan + UBSan build of the oracle over every mode."""
    import subprocess
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
    out = subprocess.run(["make", "-s", "-C", here, "asan"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "asan ok" in out.stdout, out.stdout[-2000:] + out.stderr[-2000:]


@pytest.mark.parametrize("wsz,extend", [(2, False), (3, False), (3, True), (4, False), (4, True), (5, True),
                                        (6, False), (7, True)])
def test_descriptors_unit_norm_every_window(orc, wsz, extend):
    """normalize sums every square for any nfeatures (16, 36, 72, 64, 128,
    200, 144, 392): unit L2 norm (the reference's tree reads out of bounds
    below 64 and double-adds where nfeatures is not a power of two; DESIGN.md,
    fixed semantics)."""
    img = np.load(os.path.join(GOLDEN, "images.npz"))["left_640x480"]
    p = orc.make_param(4, 4.0, upright=False, extend=extend, desc_wsz=wsz)
    pts, d, _ = orc.detect(p, img, 640, 480)
    assert len(pts) > 100 and d.shape[1] == wsz * wsz * (8 if extend else 4)
    n = np.sqrt((d.astype(np.float64) ** 2).sum(1))
    assert np.abs(n - 1).max() < 1e-5


def test_descriptor_quotient_matches_ieee_division(orc):
    """The descriptor kernels compute rpos / cpos as x * r + fma remainder
    correction (r = 1 / spacing once per keypoint, surfhip_kernels.hip
    div_by) instead of the reference's per-sample division (surfd.cu:1290-1292,
    2420-2430): the quotient must be the IEEE one, since rpos^2 + cpos^2
    indexes the Gaussian LUT."""
    import ctypes as C
    fn = orc._L.or_div_by_mismatches
    fn.restype = C.c_long
    fn.argtypes = [C.c_long, C.c_uint64]
    assert fn(20_000_000, 12345) == 0


# Surfor::init (surf.cpp:67-79), allocMemory's geometry (surf.cpp:377-392 with
# cuda_utils.h:160-163 iAlignUp) and cuFindMaximumWithInterp's NMS borders and
# grid (surfd.cu:3060-3076), compiled from the reference as they stand.

_INIT_CASES = [(m, st, d, u, e, wsz) for m in range(6, 21) for st in (1, 2, 3) for d in (False, True)
               for u, e in ((True, False), (False, True)) for wsz in (1, 2, 3, 4, 5, 6, 7)]


def _ref_init(L, noct, thresh, doubled, mask, st, upright, extend, wsz, w=1920, h=1080):
    v = np.zeros(16, np.int32)
    L.ref_surfor_init(v.ctypes.data, noct, thresh, int(doubled), mask, st, int(upright), int(extend), wsz, w, h)
    f = v.view(np.float32)
    return {"doubled": bool(v[0]), "noctaves": int(v[1]), "divisor": f[2], "init_lobe": int(v[3]),
            "max_scale": int(v[4]), "sampling": int(v[5]), "thresh": f[6], "upright": bool(v[7]),
            "extend": bool(v[8]), "desc_wsz": int(v[9]), "mag_factor": int(v[10]),
            "orient_size": int(v[11]), "nfeatures": int(v[12]), "whp": (int(v[13]), int(v[14]), int(v[15]))}


def test_param_derivation_pinned_to_reference_init(orc, surf):
    """Every SurfParam field the oracle (or_init_param) and the product
    (surfhip_make_param, host code of libsurfhip.so: no GPU call) derive,
    against Surfor::init's own statements, over init masks 6-20, sampling
    1-3, doubled, rotated/extended and desc_wsz 1-7; whp.z = iAlignUp(W, 128)
    is the pitch the ingest ring and the bench use."""
    L = _ref_or_skip(orc)
    for mask, st, d, u, e, wsz in _INIT_CASES:
        r = _ref_init(L, 4, 4.0, d, mask, st, u, e, wsz)
        o = orc.make_param(4, 4.0, d, mask, st, u, e, wsz)
        g = surf.make_param(4, 4.0, doubled=d, init_mask_size=mask, sampling_step=st, upright=u,
                            extend=e, desc_wsz=wsz)
        for name in ("doubled", "noctaves", "init_lobe", "max_scale", "sampling", "upright", "extend",
                     "desc_wsz", "mag_factor", "orient_size", "nfeatures"):
            assert getattr(o, name) == r[name] == getattr(g, name), (name, mask, st, d, u, e, wsz)
        for name in ("divisor", "thresh"):
            want = np.float32(r[name]).tobytes()
            assert np.float32(getattr(o, name)).tobytes() == want == np.float32(getattr(g, name)).tobytes()
    assert r["whp"] == (1920, 1080, surf.align_up(1920, 128))


@pytest.mark.parametrize("w,h", [(640, 480), (1920, 1080), (3840, 2160), (321, 241), (1281, 961), (64, 48)])
@pytest.mark.parametrize("mask,st,doubled,noct", [(9, 2, False, 4), (9, 2, True, 5), (6, 1, False, 6),
                                                   (12, 3, False, 4), (18, 2, True, 4), (15, 1, True, 3)])
def test_geometry_pinned_to_reference_alloc_memory(orc, w, h, mask, st, doubled, noct):
    """or_geometry's iwhp / swhps / osizes / tot_osize against allocMemory's
    own statements (the product's derive() is checked against the same
    reference values on the GPU: test_gpu_parity.py), and the oracle's NMS
    start offsets and launch extent against cuFindMaximumWithInterp's."""
    L = _ref_or_skip(orc)
    p = orc.make_param(noct, 4.0, doubled, mask, st, True, False, 4)
    g, octs = orc.geometry(p, w, h)
    iwhp = np.zeros(3, np.int32)
    sw = np.zeros(3 * 8, np.int32)
    osz = np.zeros(8, np.int32)
    tot = L.ref_alloc_geometry(int(doubled), p.sampling, p.max_scale, noct, w, h, iwhp.ctypes.data,
                               sw.ctypes.data, osz.ctypes.data)
    assert (g.iwhp.x, g.iwhp.y, g.iwhp.z) == tuple(iwhp)
    assert g.tot_osize == tot
    for o in range(noct):
        assert (g.swhp[o].x, g.swhp[o].y, g.swhp[o].z) == tuple(sw[3 * o:3 * o + 3]), o
        assert g.osize[o] == osz[o], o
        q = octs[o]
        mb = np.zeros(3, np.int32)
        grid = np.zeros(3, np.int32)
        borders = np.array(list(q.borders), np.int32)
        L.ref_nms_grid(p.max_scale, borders.ctypes.data, g.swhp[o].x, g.swhp[o].y, mb.ctypes.data, grid.ctypes.data)
        nlev = int(grid[2])
        assert nlev == len(range(1, p.max_scale - 1, 2))
        assert list(q.mborders)[:nlev] == mb[:nlev].tolist(), o
        # the oracle keeps the extent in threads (DX = DY = 16 per block)
        assert (q.nms_gx, q.nms_gy) == (int(grid[0]) * 16, int(grid[1]) * 16), o
