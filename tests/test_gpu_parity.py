"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bar (BASELINE.json north_star): integral image and Hessian planes bit-exact;
keypoint tuple (x, y, scale, octave, strength, laplace sign) bit-exact;
orientation bit-exact (deterministic reduction order on both sides);
descriptors within 1e-4 L2 per keypoint (float atomics order).
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from conftest import GOLDEN, REF_DATA, assert_points_equal, canonical, desc_l2

pytestmark = pytest.mark.gpu

DESC_TOL = 1e-4


def gpu_run(surf, param, frames, w, h, max_pts=16384, desc=True, want_ws=False, cand_cap=0):
    """Upload frames [n, H, pitch], run detect_batch, return per-frame results."""
    n, _, pitch = frames.shape
    stride = h * pitch
    det = surf.Detector(param, w, h, max_batch=n, max_pts=max_pts, cand_cap=cand_cap)
    fb = surf.DeviceBuffer(frames.nbytes)
    fb.upload(frames)
    nf = param.nfeatures
    pb = surf.DeviceBuffer(48 * n * max_pts)
    db = surf.DeviceBuffer(4 * n * max_pts * nf) if desc else None
    cb = surf.DeviceBuffer(4 * n)
    det.detect_batch(fb.ptr, n, pitch, stride, pb.ptr, db.ptr if desc else None, cb.ptr)
    surf.synchronize()
    counts = cb.download(np.int32, n)
    pts = pb.download(surf.POINT_DTYPE, n * max_pts).reshape(n, max_pts)
    ds = db.download(np.float32, n * max_pts * nf).reshape(n, max_pts, nf) if desc else None
    out = {"counts": counts, "pts": [pts[f, :counts[f]] for f in range(n)],
           "desc": [ds[f, :counts[f]] for f in range(n)] if desc else None,
           "cand": det.candidates(n), "truncated": det.truncated(), "capacity": det.capacity()}
    if want_ws:
        ii, iis, rs, rss = det.workspace()
        out["ii"] = surf.download_ptr(ii, np.int32, n * iis).reshape(n, -1)
        out["resp"] = surf.download_ptr(rs, np.float32, n * rss).reshape(n, -1)
        out["geom"] = det.geometry()
    det.close()
    return out


def compare_frame(g_pts, g_desc, o_pts, o_desc, upright):
    assert_points_equal(g_pts, o_pts)
    if not upright:
        same = g_pts["ori"].view(np.uint32) == o_pts["ori"].view(np.uint32)
        assert same.all(), f"ori differs at {int(np.argmin(same))}"
    if g_desc is not None:
        err = desc_l2(g_desc, o_desc)
        assert err.max() <= DESC_TOL, f"descriptor L2 max {err.max():.3g} at {int(err.argmax())}"


@pytest.mark.parametrize("w,h", [(64, 48), (321, 241), (640, 480), (1920, 1080)])
def test_integral_bit_exact(surf, orc, w, h):
    frames = surf.synth_frames(2, w, h)
    param = surf.make_param(4, 4.0, upright=True)
    det = surf.Detector(param, w, h, max_batch=2, max_pts=1024)
    fb = surf.DeviceBuffer(frames.nbytes)
    fb.upload(frames)
    det.run_integral(fb.ptr, 2, frames.shape[2], h * frames.shape[2])
    surf.synchronize()
    ii, iis, _, _ = det.workspace()
    got = surf.download_ptr(ii, np.int32, 2 * iis).reshape(2, h + 1, -1)
    for f in range(2):
        ref = orc.integral(frames[f], w, h)          # zero pad columns included
        np.testing.assert_array_equal(got[f], ref)
    det.close()


def test_integral_saturated_4k_wraparound(surf, orc):
    """All-255 3840x2160: the int32 image tops out at 2,115,072,000 (< 2^31) and
    getSum's pairwise adds wrap."""
    w, h = 3840, 2160
    frames = np.full((1, h, surf.align_up(w, 128)), 255, np.uint8)
    param = surf.make_param(5, 4.0, upright=True)
    det = surf.Detector(param, w, h, max_batch=1, max_pts=1024)
    fb = surf.DeviceBuffer(frames.nbytes)
    fb.upload(frames)
    det.run_integral(fb.ptr, 1, frames.shape[2], 0)
    surf.synchronize()
    ii, iis, _, _ = det.workspace()
    got = surf.download_ptr(ii, np.int32, iis).reshape(h + 1, -1)
    assert got[h, w] == 255 * w * h
    ref = orc.integral(frames[0], w, h)
    np.testing.assert_array_equal(got[:, :w + 1], ref[:, :w + 1])
    det.close()


def _plane_views(resp, g, octs, p):
    """Yield (octave, scale, plane[sh, sw]) for every plane the Hessian computes
    (planes 0/1 of octaves > 0 are the reference's halfImage copies; the HIP
    path reads them in place from octave o-1 instead of materialising them)."""
    for o in range(p.noctaves):
        sw, sh, sp = g.swhp[o].x, g.swhp[o].y, g.swhp[o].z
        for s in range(0 if o == 0 else 2, p.max_scale):
            base = g.ooff[o] + s * g.osize[o]
            yield o, s, resp[base:base + sh * sp].reshape(sh, sp)[:, :sw]


@pytest.mark.parametrize("w,h,noct", [(64, 48, 4), (333, 211, 4), (640, 480, 4), (1920, 1080, 4), (3840, 2160, 4),
                                      (3840, 2160, 5), (1920, 1080, 6), (1100, 700, 5)])
def test_hessian_planes_bit_exact(surf, orc, w, h, noct):
    """Octaves 0/1 (LDS rings), 2-4 (streaming accumulation; 4 needs 5
    octaves) and beyond (per-sample gather, the 6-octave case)."""
    frames = surf.synth_frames(1, w, h, first=7)
    param = surf.make_param(noct, 4.0, upright=True)
    res = gpu_run(surf, param, frames, w, h, want_ws=True, desc=False)
    op = orc.make_param(noct, 4.0, upright=True)
    _, ref, g, octs = orc.hessian(op, frames[0], w, h)
    got = res["resp"][0]
    for (o, s, rp), (_, _, gp) in zip(_plane_views(ref, g, octs, op), _plane_views(got, g, octs, op)):
        same = rp.view(np.uint32) == gp.view(np.uint32)
        assert same.all(), f"octave {o} scale {s}: {(~same).sum()} cells differ, first at {np.argwhere(~same)[0]}"


def _extreme_frame(kind, w, h, pitch):
    """Frames that drive the box sums to their extremes: every value the
    Hessian kernels hold must stay an exact integer (k_hess_q0 keeps them in
    fp32 below 2^24 by rebasing its local integral)."""
    rng = np.random.default_rng(5)
    f = np.zeros((h, pitch), np.uint8)
    if kind == "white":
        f[:, :w] = 255
    elif kind == "noise":
        f[:, :w] = rng.integers(0, 256, (h, w), dtype=np.uint8)
    elif kind == "vstripes":       # 0/255 columns of period 6: large dxx, zero dyy
        f[:, :w] = np.where((np.arange(w) // 3) % 2 == 0, 255, 0).astype(np.uint8)[None, :]
    elif kind in ("hbands", "vbands"):
        # random-width bands varying along one axis only: one of sxx / syy is
        # an exact 0 while the other takes both signs and sxy = 0, so the
        # product's -0 / +0 (the reference's (float)int conversions) must
        # come out bit for bit
        n = h if kind == "hbands" else w
        edges = np.cumsum(rng.integers(3, 40, n))
        band = np.searchsorted(edges, np.arange(n), side="right")
        vals = rng.integers(0, 256, band.max() + 1, dtype=np.uint8)[band]
        f[:, :w] = vals[:, None] if kind == "hbands" else vals[None, :]
    elif kind == "checker":        # 7x5 blocks: large dxy
        yy, xx = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
        f[:, :w] = np.where(((yy // 5) + (xx // 7)) % 2 == 0, 255, 0).astype(np.uint8)
    return f


@pytest.mark.parametrize("kind", ["white", "noise", "vstripes", "checker", "hbands", "vbands"])
@pytest.mark.parametrize("env", ["SURFHIP_HESS_W=1", "SURFHIP_HESS_W=0", "SURFHIP_P0=0", "SURFHIP_P0=95",
                                 "SURFHIP_HESS_GATHER=1"])
def test_hessian_planes_extreme_frames(surf, orc, monkeypatch, kind, env):
    w, h = 1920, 1080
    name, _, val = env.partition("=")
    monkeypatch.setenv(name, val)
    frames = _extreme_frame(kind, w, h, surf.align_up(w, 128))[None]
    param = surf.make_param(4, 4.0, upright=True)
    res = gpu_run(surf, param, frames, w, h, want_ws=True, desc=False)
    op = orc.make_param(4, 4.0, upright=True)
    _, ref, g, octs = orc.hessian(op, frames[0], w, h)
    got = res["resp"][0]
    for (o, s, rp), (_, _, gp) in zip(_plane_views(ref, g, octs, op), _plane_views(got, g, octs, op)):
        same = rp.view(np.uint32) == gp.view(np.uint32)
        assert same.all(), f"{kind}/{env}: octave {o} scale {s}: {(~same).sum()} cells differ"


@pytest.mark.parametrize("env", ["SURFHIP_HESS_W=0", "SURFHIP_HESS_W=0,SURFHIP_Q01=0", "SURFHIP_HESS_GATHER=1",
                                 "SURFHIP_HESS_GATHER=1,SURFHIP_HESS_T0=0", "SURFHIP_P0=0", "SURFHIP_P0=95", "SURFHIP_P0=92", "SURFHIP_P0=91", "SURFHIP_P0=32"])
@pytest.mark.parametrize("w,h,noct", [(640, 480, 4), (1920, 1080, 4), (1920, 1080, 2), (960, 540, 3)])
def test_hessian_alternate_kernels_bit_exact(surf, orc, monkeypatch, env, w, h, noct):
    """The selectable Hessian plans give the same planes: k_hess_q1 (alone or
    merged with k_hess_q0 in k_hess_q01) + the gather kernel instead of
    k_hess_w, the gather plan (octave 0 from LDS tiles, k_hessian_t0, or every
    octave on k_hessian), octave 0 on k_hess_q0 instead of k_hess_p0
    and k_hess_p0 with 3-step barrier intervals; 2 octaves (no k_hess_w) and 3 octaves
    (k_hess_w with octaves 1-2).  The plan reads these switches when a
    detector is created."""
    for kv in env.split(","):
        name, _, val = kv.partition("=")
        monkeypatch.setenv(name, val or "1")
    frames = surf.synth_frames(1, w, h, first=21)
    param = surf.make_param(noct, 4.0, upright=True)
    res = gpu_run(surf, param, frames, w, h, want_ws=True, desc=False)
    op = orc.make_param(noct, 4.0, upright=True)
    _, ref, g, octs = orc.hessian(op, frames[0], w, h)
    got = res["resp"][0]
    for (o, s, rp), (_, _, gp) in zip(_plane_views(ref, g, octs, op), _plane_views(got, g, octs, op)):
        same = rp.view(np.uint32) == gp.view(np.uint32)
        assert same.all(), f"{env}: octave {o} scale {s}: {(~same).sum()} cells differ"


@pytest.mark.parametrize("upright,extend", [(True, False), (False, False), (True, True), (False, True)])
def test_detect_describe_synthetic(surf, orc, upright, extend):
    w, h = 640, 480
    frames = surf.synth_frames(3, w, h, first=100)
    param = surf.make_param(4, 4.0, upright=upright, extend=extend)
    res = gpu_run(surf, param, frames, w, h)
    op = orc.make_param(4, 4.0, upright=upright, extend=extend)
    for f in range(3):
        o_pts, o_desc, nc = orc.detect(op, frames[f], w, h)
        assert res["cand"][f] == nc
        compare_frame(res["pts"][f], res["desc"][f], o_pts, o_desc, upright)


@pytest.mark.parametrize("cube", ["0", "1"])
def test_fit_records_from_scan(surf, orc, monkeypatch, cube):
    """k_nms_fit's first pass from the scan's record of the 19 responses
    (SURFHIP_FIT_CUBE=1, the default for batches > 8) or from the planes
    (=0, the small-batch default): the same keypoints, bit for bit."""
    monkeypatch.setenv("SURFHIP_FIT_CUBE", cube)
    w, h = 640, 480
    frames = surf.synth_frames(3, w, h, first=300)
    param = surf.make_param(4, 4.0, upright=True)
    res = gpu_run(surf, param, frames, w, h)
    op = orc.make_param(4, 4.0, upright=True)
    for f in range(3):
        o_pts, o_desc, nc = orc.detect(op, frames[f], w, h)
        assert res["cand"][f] == nc
        compare_frame(res["pts"][f], res["desc"][f], o_pts, o_desc, True)


@pytest.mark.parametrize("trace_desc,desc", [("1", True), ("0", True), ("1", False)])
def test_laplace_in_fit_or_describe(surf, orc, monkeypatch, trace_desc, desc):
    """makePoint's laplace (getTrace, surfd.cu:369-377, 1010-1020) taken in
    k_describe_u2 from the fit's stashed inputs (SURFHIP_TRACE_DESC=1, the
    default when k_describe_u2 runs), in k_nms_fit (=0), and in the fit when
    no descriptors are asked for: every point field equals the oracle's,
    laplace and ori (0) included, bit for bit."""
    monkeypatch.setenv("SURFHIP_TRACE_DESC", trace_desc)
    w, h = 640, 480
    frames = surf.synth_frames(12, w, h, first=700)
    param = surf.make_param(4, 4.0, upright=True)
    res = gpu_run(surf, param, frames, w, h, desc=desc)
    op = orc.make_param(4, 4.0, upright=True)
    for f in (0, 5, 11):
        o_pts, o_desc, nc = orc.detect(op, frames[f], w, h)
        assert res["cand"][f] == nc
        assert_points_equal(res["pts"][f], o_pts)
        assert (res["pts"][f]["ori"] == 0).all()
        assert set(np.unique(res["pts"][f]["laplace"])) <= {-1, 1}
        if desc:
            compare_frame(res["pts"][f], res["desc"][f], o_pts, o_desc, True)


@pytest.mark.parametrize("extend", [False, True])
@pytest.mark.parametrize("atomic", [False, True])
def test_rotated_descriptor_kernels(surf, orc, monkeypatch, extend, atomic):
    """Rotated 4x4 descriptors: the atomic-free floor-cell kernel (default,
    k_describe_rot) and the LDS-atomic kernel (SURFHIP_ROT_ATOMIC) against the
    oracle; the atomic-free one is also run twice and must repeat bit for bit."""
    if atomic:
        monkeypatch.setenv("SURFHIP_ROT_ATOMIC", "1")
    w, h = 1280, 720
    frames = surf.synth_frames(2, w, h, first=300)
    param = surf.make_param(5, 4.0, upright=False, extend=extend)
    res = gpu_run(surf, param, frames, w, h)
    op = orc.make_param(5, 4.0, upright=False, extend=extend)
    for f in range(2):
        o_pts, o_desc, _ = orc.detect(op, frames[f], w, h)
        assert len(o_pts) > 100
        compare_frame(res["pts"][f], res["desc"][f], o_pts, o_desc, False)
    if not atomic:
        again = gpu_run(surf, param, frames, w, h)
        for f in range(2):
            assert again["desc"][f].tobytes() == res["desc"][f].tobytes()


@pytest.mark.parametrize("upright", [True, False])
def test_single_frame_gather_plan(surf, orc, monkeypatch, upright):
    """Config #2 as a single-frame detector (max_batch 1) on its default plan:
    every octave on the gather Hessian kernel; keypoints/descriptors as the oracle."""
    monkeypatch.delenv("SURFHIP_HESS_GATHER", raising=False)
    w, h = 1920, 1080
    frames = surf.synth_frames(1, w, h, first=7)
    param = surf.make_param(4, 4.0, upright=upright)
    res = gpu_run(surf, param, frames, w, h)
    op = orc.make_param(4, 4.0, upright=upright)
    o_pts, o_desc, nc = orc.detect(op, frames[0], w, h)
    assert res["cand"][0] == nc
    compare_frame(res["pts"][0], res["desc"][0], o_pts, o_desc, upright)


@pytest.mark.parametrize("index", [0, 56])
def test_detect_describe_1080p(surf, orc, index):
    """Config #2: single 1920x1080, 4 octaves, 64-D, upright (main.cpp:187-204).
    Frame 56 holds a keypoint whose getTrace box reaches column -1 (the
    reference's unchecked flat read, see trace_sign)."""
    w, h = 1920, 1080
    frames = surf.synth_frames(1, w, h, first=index)
    param = surf.make_param(4, 4.0, upright=True)
    res = gpu_run(surf, param, frames, w, h)
    op = orc.make_param(4, 4.0, upright=True)
    o_pts, o_desc, _ = orc.detect(op, frames[0], w, h)
    assert len(o_pts) > 1000
    assert set(np.unique(o_pts["o"])) == {0, 1, 2, 3}
    compare_frame(res["pts"][0], res["desc"][0], o_pts, o_desc, True)


@pytest.mark.skipif(not os.path.exists(os.path.join(GOLDEN, "left_1280x960_upright.npz")),
                    reason="golden fixtures not generated")
@pytest.mark.parametrize("name", ["left_1280x960_upright", "left_1280x960_rotated", "right_1280x960_upright",
                                  "left_640x480_upright", "left_1280x960_rotated_ext"])
def test_golden_fixtures(surf, name):
    """data/left.pgm / right.pgm (the reference's only data) vs frozen oracle outputs."""
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    img = np.load(os.path.join(GOLDEN, "images.npz"))[str(z["image_key"])]
    h, w = img.shape
    meta = z["meta"]
    upright, extend = bool(meta[0]), bool(meta[1])
    pitch = surf.align_up(w, 128)
    frames = np.zeros((1, h, pitch), np.uint8)
    frames[0, :, :w] = img
    param = surf.make_param(4, 4.0, upright=upright, extend=extend)
    res = gpu_run(surf, param, frames, w, h)
    pts = np.frombuffer(z["points"].tobytes(), dtype=surf.POINT_DTYPE)
    compare_frame(res["pts"][0], res["desc"][0], pts, z["desc"], upright)


def test_batch_equals_single(surf):
    """Frames processed in one batch give the same results as one at a time."""
    w, h = 320, 240
    frames = surf.synth_frames(4, w, h, first=55)
    param = surf.make_param(4, 4.0, upright=False)
    batch = gpu_run(surf, param, frames, w, h)
    for f in range(4):
        one = gpu_run(surf, param, frames[f:f + 1], w, h)
        assert_points_equal(one["pts"][0], batch["pts"][f], fields=("x", "y", "scale", "o", "strength", "laplace", "ori"))
        assert desc_l2(one["desc"][0], batch["desc"][f]).max() <= DESC_TOL


def test_max_pts_cap_keeps_canonical_prefix(surf, orc):
    w, h = 640, 480
    frames = surf.synth_frames(1, w, h, first=3)
    param = surf.make_param(4, 4.0, upright=True)
    full = gpu_run(surf, param, frames, w, h, max_pts=16384)
    cap = max(1, len(full["pts"][0]) // 3)
    part = gpu_run(surf, param, frames, w, h, max_pts=cap)
    assert part["counts"][0] == cap
    assert_points_equal(part["pts"][0], full["pts"][0][:cap])
    op = orc.make_param(4, 4.0, upright=True)
    o_pts, _, _ = orc.detect(op, frames[0], w, h, max_pts=cap, desc=False)
    assert_points_equal(part["pts"][0], o_pts)


def test_flat_and_tiny_frames(surf):
    """Edge cases: a constant frame yields no keypoints; a tiny frame works."""
    param = surf.make_param(4, 4.0, upright=True)
    flat = np.full((2, 96, 128), 77, np.uint8)
    r = gpu_run(surf, param, flat, 100, 96)
    assert (r["counts"] == 0).all()
    tiny = surf.synth_frames(1, 40, 36)
    r = gpu_run(surf, param, tiny, 40, 36)
    assert r["counts"][0] >= 0


def test_surfor_mirror_api(surf, orc):
    """The reference-shaped API (Surfor.init / detectAndCompute, surf.h)."""
    w, h = 640, 480
    frame = surf.synth_frames(1, w, h, first=11)[0]
    d = surf.Surfor()
    d.init(4, 4.0, False, 9, 2, True, False, 4, w, h)
    data = surf.initSurfData(10000, True, True)
    img = surf.DeviceBuffer(frame.nbytes)
    img.upload(frame)
    dptr = d.detectAndCompute(img.ptr, data, (w, h, frame.shape[1]), True)
    op = orc.make_param(4, 4.0, upright=True)
    o_pts, o_desc, _ = orc.detect(op, frame, w, h)
    assert data.num_pts == len(o_pts)
    assert_points_equal(data.h_data[:data.num_pts], o_pts)
    got = surf.download_ptr(dptr, np.float32, data.num_pts * 64).reshape(-1, 64)
    assert desc_l2(got, o_desc).max() <= DESC_TOL
    surf.check(surf.lib.surfhip_free(dptr))
    surf.freeSurfData(data)


# ------------------------------------------------------------------ match
MATCH_FIELDS = ("score", "match", "match_x", "match_y", "ambiguity")


def gpu_match(surf, p1, p2, f1, f2, flags=0, own_scratch=False):
    n1, n2 = len(p1), len(p2)
    nf = f1.shape[1]
    b1 = surf.DeviceBuffer(max(48 * n1, 48))
    b2 = surf.DeviceBuffer(max(48 * n2, 48))
    d1 = surf.DeviceBuffer(max(f1.nbytes, 4))
    d2 = surf.DeviceBuffer(max(f2.nbytes, 4))
    if n1:
        b1.upload(np.ascontiguousarray(p1))
        d1.upload(np.ascontiguousarray(f1))
    if n2:
        b2.upload(np.ascontiguousarray(p2))
        d2.upload(np.ascontiguousarray(f2))
    scratch = None
    if own_scratch:
        scratch = surf.DeviceBuffer(max(surf.match_scratch_bytes(n1, n2, flags), 4))
    surf.match_points(b1.ptr, b2.ptr, d1.ptr, d2.ptr, n1, n2, nf, flags, scratch.ptr if scratch else None)
    surf.synchronize()
    return b1.download(surf.POINT_DTYPE, n1) if n1 else np.zeros(0, surf.POINT_DTYPE)


def assert_match_equal(got, ref):
    for f in MATCH_FIELDS:
        g, r = got[f], ref[f]
        if g.dtype == np.float32:
            g, r = g.view(np.uint32), r.view(np.uint32)
        bad = np.nonzero(g != r)[0]
        assert len(bad) == 0, f"{f} differs at {bad[:5]}"


@pytest.mark.parametrize("tag,flags", [("ref", 0), ("full", 1)])
def test_match_golden_left_right(surf, orc, tag, flags):
    """Surfor::match of the reference's own image pair (main.cpp:250),
    bit-exact against the committed oracle vectors."""
    z = np.load(os.path.join(GOLDEN, "match_left_right_upright.npz"))
    a = np.load(os.path.join(GOLDEN, "left_1280x960_upright.npz"))
    b = np.load(os.path.join(GOLDEN, "right_1280x960_upright.npz"))
    p1, p2 = a["points"].view(surf.POINT_DTYPE), b["points"].view(surf.POINT_DTYPE)
    got = gpu_match(surf, p1, p2, a["desc"], b["desc"], flags)
    ref = np.zeros(len(p1), surf.POINT_DTYPE)
    for f in MATCH_FIELDS:
        ref[f] = z[f"{tag}_{f}"]
    assert_match_equal(got, ref)
    # the detect fields are left untouched
    for f in ("x", "y", "scale", "strength", "laplace"):
        np.testing.assert_array_equal(got[f], p1[f])


@pytest.mark.parametrize("n1,n2,nf,flags", [(1, 0, 64, 0), (7, 31, 64, 0), (7, 31, 64, 1), (300, 545, 64, 0),
                                             (300, 545, 64, 1), (1000, 4096, 64, 0), (3000, 3000, 64, 1),
                                             (257, 700, 128, 0), (129, 333, 36, 1), (64, 64, 16, 0),
                                             (200, 333, 200, 0), (70, 90, 392, 1)])
def test_match_random_vs_oracle(surf, orc, n1, n2, nf, flags):
    rng = np.random.default_rng(n1 + 7 * n2 + nf + flags)
    f1 = rng.standard_normal((n1, nf)).astype(np.float32)
    f2 = rng.standard_normal((n2, nf)).astype(np.float32)
    f1 /= np.linalg.norm(f1, axis=1, keepdims=True)
    if n2:
        f2 /= np.linalg.norm(f2, axis=1, keepdims=True)
        f2[n2 // 2] = f1[0]                          # a perfect partner (ties across rows)
    p1 = np.zeros(n1, surf.POINT_DTYPE)
    p1["x"] = rng.uniform(0, 100, n1)
    p2 = np.zeros(n2, surf.POINT_DTYPE)
    p2["x"] = rng.uniform(0, 1920, n2)
    p2["y"] = rng.uniform(0, 1080, n2)
    got = gpu_match(surf, p1, p2, f1, f2, flags, own_scratch=(n1 == 300))
    ref = orc.match(p1, p2, f1, f2, full_tail=bool(flags))
    assert_match_equal(got, ref)


def test_surfor_match_end_to_end(surf, orc):
    """Surfor.init -> detectAndCompute(left), detectAndCompute(right) ->
    match (main.cpp:236-250) through the reference-shaped mirror."""
    a = np.load(os.path.join(GOLDEN, "images.npz"))
    d = surf.Surfor()
    w, h = 1280, 960
    d.init(4, 4.0, False, 9, 2, True, False, 4, w, h)
    out = []
    for key in ("left_1280x960", "right_1280x960"):
        img = a[key]
        data = surf.initSurfData(10000, True, True)
        buf = surf.DeviceBuffer(img.nbytes)
        buf.upload(img)
        dptr = d.detectAndCompute(buf.ptr, data, (w, h, img.shape[1]), True)
        out.append((data, dptr, buf))
    (d1, f1, _), (d2, f2, _) = out
    d.match(d1, d2, f1, f2)
    z = np.load(os.path.join(GOLDEN, "match_left_right_upright.npz"))
    # the GPU descriptors agree with the oracle's within 1e-4 L2, so scores
    # may differ in the last bits; indices must agree where the best is clear
    assert d1.num_pts == len(z["ref_match"])
    got = d1.h_data[:d1.num_pts]
    g1 = surf.download_ptr(f1, np.float32, d1.num_pts * 64).reshape(-1, 64)
    g2 = surf.download_ptr(f2, np.float32, d2.num_pts * 64).reshape(-1, 64)
    pts2 = surf.download_ptr(d2.d_data.ptr, surf.POINT_DTYPE, d2.num_pts)
    ref = orc.match(got, pts2, g1, g2)                # oracle on the GPU's own descriptors: bit-exact
    assert_match_equal(got, ref)
    clear = z["ref_ambiguity"] < 0.99
    assert (got["match"][clear] == z["ref_match"][clear]).mean() > 0.99
    for data, dptr, _ in out:
        surf.check(surf.lib.surfhip_free(dptr))
        surf.freeSurfData(data)


# ---------------------------------------------------------- doubled image
@pytest.mark.parametrize("w,h", [(64, 48), (333, 211), (1920, 1080)])
def test_doubled_integral_and_planes_bit_exact(surf, orc, w, h):
    """doubled = true (surf.cpp:234-235, cuIntegralDoubleU4 surfd.cu:2707-2772):
    the (2W-1) x (2H-1) integral image and every response plane."""
    frames = surf.synth_frames(2, w, h, first=31)
    param = surf.make_param(4, 4.0, doubled=True, upright=True)
    res = gpu_run(surf, param, frames, w, h, want_ws=True, desc=False)
    op = orc.make_param(4, 4.0, doubled=True, upright=True)
    for f in range(2):
        ii, ref, g, octs = orc.hessian(op, frames[f], w, h)
        assert (g.iwhp.x, g.iwhp.y) == (2 * w - 1, 2 * h - 1)
        got_ii = res["ii"][f][:ii.size].reshape(ii.shape)
        np.testing.assert_array_equal(got_ii, ii)
        got = res["resp"][f]
        for (o, s, rp), (_, _, gp) in zip(_plane_views(ref, g, octs, op), _plane_views(got, g, octs, op)):
            same = rp.view(np.uint32) == gp.view(np.uint32)
            assert same.all(), f"octave {o} scale {s}: {(~same).sum()} cells differ"


@pytest.mark.parametrize("upright,extend", [(True, False), (False, False), (True, True)])
def test_doubled_detect_describe(surf, orc, upright, extend):
    w, h = 640, 480
    frames = surf.synth_frames(2, w, h, first=140)
    param = surf.make_param(4, 4.0, doubled=True, upright=upright, extend=extend)
    res = gpu_run(surf, param, frames, w, h)
    op = orc.make_param(4, 4.0, doubled=True, upright=upright, extend=extend)
    for f in range(2):
        o_pts, o_desc, nc = orc.detect(op, frames[f], w, h)
        assert res["cand"][f] == nc and nc > 100
        compare_frame(res["pts"][f], res["desc"][f], o_pts, o_desc, upright)


def test_doubled_reference_image(surf, orc):
    """The reference's 640x480 left image with doubled = true."""
    img = np.load(os.path.join(GOLDEN, "images.npz"))["left_640x480"]
    w, h = 640, 480
    frames = np.zeros((1, h, 640), np.uint8)
    frames[0] = img
    param = surf.make_param(4, 4.0, doubled=True, upright=True)
    res = gpu_run(surf, param, frames, w, h)
    op = orc.make_param(4, 4.0, doubled=True, upright=True)
    o_pts, o_desc, nc = orc.detect(op, img, w, h)
    assert res["cand"][0] == nc
    compare_frame(res["pts"][0], res["desc"][0], o_pts, o_desc, True)


@pytest.mark.parametrize("depth,upright,extend", [(1, True, False), (2, True, False), (3, True, False),
                                                  (2, False, True)])
def test_ingest_ring_equals_resident_batches(surf, depth, upright, extend, tmp_path):
    """Pinned-host ingest ring (surfhip_ingest_*): five batches (last one
    ragged) through a ring of `depth` slots give slabs byte-identical to
    detect_batch + pack_slab on the same frames resident in HBM; the
    keypoint file written from them reads back the same."""
    w, h, B, max_pts = 320, 240, 3, 4096
    param = surf.make_param(4, 4.0, False, 9, 2, upright, extend, 4)
    nf = param.nfeatures
    sizes = [3, 3, 2, 3, 1]
    frames = surf.synth_frames(sum(sizes), w, h, first=40)
    n_all, _, pitch = frames.shape
    # resident reference: one batch at a time, packed
    ref = []
    det = surf.Detector(param, w, h, max_batch=B, max_pts=max_pts)
    fb, pb = surf.DeviceBuffer(frames[:B].nbytes), surf.DeviceBuffer(48 * B * max_pts)
    db, cb = surf.DeviceBuffer(4 * B * max_pts * nf), surf.DeviceBuffer(4 * B)
    first = 0
    for n in sizes:
        fb.upload(np.ascontiguousarray(frames[first:first + n]))
        det.detect_batch(fb.ptr, n, pitch, h * pitch, pb.ptr, db.ptr, cb.ptr)
        total = det.batch_total(n)
        sb = surf.DeviceBuffer(det.slab_bytes(n, total))
        det.pack_slab(pb.ptr, db.ptr, cb.ptr, n, sb.ptr)
        surf.synchronize()
        ref.append(sb.download(np.uint8, det.slab_bytes(n, total)))
        first += n
    det.close()
    det = surf.Detector(param, w, h, max_batch=B, max_pts=max_pts)
    ing = surf.Ingest(det, depth)
    got, first, path = [], 0, str(tmp_path / "ring.surfkpd")
    for n in sizes:
        if ing.pending() == depth:
            got.append(ing.collect())
        slot = ing.acquire()
        assert slot.shape[1:] == (h, surf.align_up(w, 128))
        slot[:n, :, :w] = frames[first:first + n, :, :w]
        ing.submit(n)
        first += n
    while ing.pending():
        got.append(ing.collect())
    assert len(got) == len(ref)
    for i, (g, r) in enumerate(zip(got, ref)):
        assert g.tobytes() == r.tobytes(), f"batch {i} slab differs"
        surf.dump_append(path, g, w, h, param, first_frame=sum(sizes[:i]))
    back = surf.read_dump(path)
    for (hdr, c, p, d), r in zip(back, ref):
        c0, p0, d0 = surf.parse_slab(r)
        np.testing.assert_array_equal(c, c0)
        assert p.tobytes() == p0.tobytes() and d.tobytes() == d0.tobytes()
    ing.close()
    det.close()


@pytest.mark.parametrize("w,h,mask,st,doubled,noct", [(1920, 1080, 9, 2, False, 4), (640, 480, 9, 2, True, 5),
                                                       (321, 241, 6, 1, False, 6), (3840, 2160, 12, 3, False, 4)])
def test_detector_geometry_pinned_to_reference_alloc_memory(surf, orc, w, h, mask, st, doubled, noct):
    """The product's derive() (surfhip_detector_geometry) against allocMemory's
    own statements (surf.cpp:377-392, compiled from the reference into
    oracle/_ref by oracle/ref_extract.py): iwhp, swhps and osizes."""
    L = orc.ref_host()
    if L is None:
        pytest.skip("oracle/_ref not built (no reference sources when it was built)")
    p = orc.make_param(noct, 4.0, doubled, mask, st, True, False, 4)
    iwhp = np.zeros(3, np.int32)
    sw = np.zeros(3 * 8, np.int32)
    osz = np.zeros(8, np.int32)
    L.ref_alloc_geometry(int(doubled), p.sampling, p.max_scale, noct, w, h, iwhp.ctypes.data, sw.ctypes.data,
                         osz.ctypes.data)
    param = surf.make_param(noct, 4.0, doubled=doubled, init_mask_size=mask, sampling_step=st, upright=True)
    det = surf.Detector(param, w, h, max_batch=1, max_pts=64)
    giw, gsw, _, gos = det.geometry()
    det.close()
    assert giw == tuple(iwhp)
    for o in range(noct):
        assert gsw[o] == tuple(sw[3 * o:3 * o + 3]) and gos[o] == osz[o], o


def test_detect_batch_next_equals_detect_batch(surf):
    """surfhip_detect_batch_next (the next batch's integral computed beside
    this batch's describe): over a sequence of batches -- the prefetch used
    (same next frames), not used (another batch comes instead), a ragged
    batch and a plain detect_batch in between -- every batch's keypoints and
    descriptors are byte-identical to a detect_batch of the same frames."""
    w, h, n = 640, 480, 12
    frames = [surf.synth_frames(n, w, h, first=k * 100) for k in range(3)]
    pitch = frames[0].shape[2]
    stride = h * pitch
    param = surf.make_param(4, 4.0, upright=True)
    max_pts = 4096
    bufs = []
    for fr in frames:
        b = surf.DeviceBuffer(fr.nbytes)
        b.upload(fr)
        bufs.append(b)
    pb = surf.DeviceBuffer(48 * n * max_pts)
    db = surf.DeviceBuffer(4 * n * max_pts * 64)
    cb = surf.DeviceBuffer(4 * n)

    def result(det_call, nf):
        det_call()
        surf.synchronize()
        c = cb.download(np.int32, nf)
        p = pb.download(surf.POINT_DTYPE, nf * max_pts).reshape(nf, max_pts)
        d = db.download(np.float32, nf * max_pts * 64).reshape(nf, max_pts, 64)
        return [(p[f, :c[f]].tobytes(), d[f, :c[f]].tobytes()) for f in range(nf)]

    ref = surf.Detector(param, w, h, max_batch=n, max_pts=max_pts)
    want = {}
    for k in range(3):
        for nf in (n, 7):
            want[(k, nf)] = result(lambda: ref.detect_batch(bufs[k].ptr, nf, pitch, stride, pb.ptr, db.ptr, cb.ptr),
                                   nf)
    ref.close()
    det = surf.Detector(param, w, h, max_batch=n, max_pts=max_pts)
    # (batch, nframes, next batch or None, next nframes)
    seq = [(0, n, 1, n), (1, n, 2, n), (0, n, 0, 7), (0, 7, 2, n), (2, n, None, 0), (1, n, 1, n), (1, n, 0, n),
           (0, n, None, 0)]
    for k, nf, nx, nnf in seq:
        if nx is None:
            got = result(lambda: det.detect_batch(bufs[k].ptr, nf, pitch, stride, pb.ptr, db.ptr, cb.ptr), nf)
        else:
            got = result(lambda: det.detect_batch_next(bufs[k].ptr, nf, pitch, stride, pb.ptr, db.ptr, cb.ptr,
                                                       bufs[nx].ptr, nnf, pitch, stride), nf)
        assert got == want[(k, nf)], (k, nf, nx, nnf)
    det.close()


def test_profiled_call_after_pipelined_call(surf):
    """A pipelined call leaves the next batch's integral running on the side
    stream (sharing the colsum scratch); a stage-profiled call queued right
    after it (no host sync in between) must wait for it, and
    surfhip_detector_drain keeps the prefetch valid: every result equals a
    plain detect_batch of the same frames."""
    w, h, n = 1920, 1080, 16
    frames = [surf.synth_frames(n, w, h, first=k * 50) for k in range(3)]
    pitch = frames[0].shape[2]
    stride = h * pitch
    param = surf.make_param(4, 4.0, upright=True)
    max_pts = 8192
    bufs = []
    for fr in frames:
        b = surf.DeviceBuffer(fr.nbytes)
        b.upload(fr)
        bufs.append(b)
    pb = surf.DeviceBuffer(48 * n * max_pts)
    db = surf.DeviceBuffer(4 * n * max_pts * 64)
    cb = surf.DeviceBuffer(4 * n)

    def fetch():
        surf.synchronize()
        c = cb.download(np.int32, n)
        p = pb.download(surf.POINT_DTYPE, n * max_pts).reshape(n, max_pts)
        d = db.download(np.float32, n * max_pts * 64).reshape(n, max_pts, 64)
        return [(p[f, :c[f]].tobytes(), d[f, :c[f]].tobytes()) for f in range(n)]

    ref = surf.Detector(param, w, h, max_batch=n, max_pts=max_pts)
    want = []
    for k in range(3):
        ref.detect_batch(bufs[k].ptr, n, pitch, stride, pb.ptr, db.ptr, cb.ptr)
        want.append(fetch())
    ref.close()
    det = surf.Detector(param, w, h, max_batch=n, max_pts=max_pts)
    det.detect_batch_next(bufs[0].ptr, n, pitch, stride, pb.ptr, db.ptr, cb.ptr, bufs[1].ptr, n, pitch, stride)
    det.set_profiling(True)
    det.detect_batch(bufs[2].ptr, n, pitch, stride, pb.ptr, db.ptr, cb.ptr)
    assert fetch() == want[2]
    assert det.stage_times()["total"] > 0
    det.set_profiling(False)
    det.detect_batch_next(bufs[0].ptr, n, pitch, stride, pb.ptr, db.ptr, cb.ptr, bufs[1].ptr, n, pitch, stride)
    assert fetch() == want[0]
    det.drain()
    det.detect_batch_next(bufs[1].ptr, n, pitch, stride, pb.ptr, db.ptr, cb.ptr, None, 0, 0, 0)
    assert fetch() == want[1]
    det.close()
