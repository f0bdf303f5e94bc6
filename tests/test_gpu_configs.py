"""GPU parity at the configurations the bench and BASELINE.json run.

- config #3: one 256-frame 1920x1080 batch (the bench's workload, streaming
  Hessian plan, XCD frame mapping) -- frames 0, 7, 8, 127, 255 against the
  oracle, and every frame against a single-frame detector (whose default plan
  is the gather Hessian: a second, independent path);
- config #5: 3840x2160, 5 octaves, rotated, 128-D extended, as an 8-frame
  batch -- keypoints and ori bit-exact, descriptors within 1e-4 L2;
- the candidate sort beyond the LDS capacity (> 16,384 candidates, global
  scratch path) and deterministic truncation at a small candidate capacity;
- descriptor windows other than 4 (the generic k_describe);
- the single-frame gather plan on the doubled, 5/6-octave and rotated cases.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import assert_points_equal, desc_l2
from test_gpu_parity import DESC_TOL, compare_frame, gpu_run

pytestmark = pytest.mark.gpu

W3, H3 = 1920, 1080


@pytest.fixture(scope="module")
def config3(surf):
    frames = surf.synth_frames(256, W3, H3, first=0)
    param = surf.make_param(4, 4.0, upright=True)
    res = gpu_run(surf, param, frames, W3, H3, max_pts=8192)
    return frames, res


@pytest.mark.parametrize("f", [0, 7, 8, 127, 255])
def test_config3_batch256_vs_oracle(orc, config3, f):
    frames, res = config3
    op = orc.make_param(4, 4.0, upright=True)
    o_pts, o_desc, nc = orc.detect(op, frames[f], W3, H3, max_pts=8192)
    assert len(o_pts) > 1000
    assert res["cand"][f] == nc
    compare_frame(res["pts"][f], res["desc"][f], o_pts, o_desc, True)


def test_config3_batch256_vs_single_frame(surf, monkeypatch, config3):
    """All 256 frames of the batch against a max_batch=1 detector, whose
    default plan puts every octave on the gather Hessian kernel."""
    frames, res = config3
    monkeypatch.delenv("SURFHIP_HESS_GATHER", raising=False)
    param = surf.make_param(4, 4.0, upright=True)
    max_pts = 8192
    det = surf.Detector(param, W3, H3, max_batch=1, max_pts=max_pts)
    pitch = frames.shape[2]
    fb = surf.DeviceBuffer(frames[0].nbytes)
    pb = surf.DeviceBuffer(48 * max_pts)
    db = surf.DeviceBuffer(4 * max_pts * 64)
    cb = surf.DeviceBuffer(4)
    assert not res["truncated"]
    for f in range(256):
        fb.upload(frames[f])
        det.detect_batch(fb.ptr, 1, pitch, 0, pb.ptr, db.ptr, cb.ptr)
        surf.synchronize()
        n = int(cb.download(np.int32, 1)[0])
        assert n == res["counts"][f], f
        pts = pb.download(surf.POINT_DTYPE, max_pts)[:n]
        assert_points_equal(pts, res["pts"][f])
        d = db.download(np.float32, max_pts * 64).reshape(max_pts, 64)[:n]
        assert d.tobytes() == res["desc"][f].tobytes(), f
    det.close()


def test_config3_describe_u2_deterministic(surf, monkeypatch, config3):
    """k_describe_u2 (LDS-DMA ring, the default) on the 256-frame batch: a
    second run bit-identical to the first (its ring once raced: a slot
    refilled while its reads were pending gave a few run-dependent
    descriptors per batch), and every frame within the descriptor tolerance
    of round 3's k_describe_ur (SURFHIP_DESC_UR=1; same keypoints, the two
    sum in different orders)."""
    frames, res = config3
    param = surf.make_param(4, 4.0, upright=True)
    again = gpu_run(surf, param, frames, W3, H3, max_pts=8192)
    monkeypatch.setenv("SURFHIP_DESC_UR", "1")
    ur = gpu_run(surf, param, frames, W3, H3, max_pts=8192)
    for f in range(frames.shape[0]):
        assert again["counts"][f] == res["counts"][f] == ur["counts"][f], f
        assert again["desc"][f].tobytes() == res["desc"][f].tobytes(), f
        assert desc_l2(ur["desc"][f], res["desc"][f]).max() <= DESC_TOL, f


def test_small_batch_default_plan(surf, orc, monkeypatch):
    """The plan a detector of <= 8 frames picks by default (config #2): the
    gather Hessian with octave 0 from LDS tiles, fit records, k_describe_ur --
    keypoints bit-exact and descriptors within tolerance of the oracle."""
    monkeypatch.delenv("SURFHIP_HESS_GATHER", raising=False)
    monkeypatch.delenv("SURFHIP_DESC_UR", raising=False)
    monkeypatch.delenv("SURFHIP_FIT_CUBE", raising=False)
    w, h = 1920, 1080
    frames = surf.synth_frames(2, w, h, first=900)
    param = surf.make_param(4, 4.0, upright=True)
    res = gpu_run(surf, param, frames, w, h, max_pts=8192)
    op = orc.make_param(4, 4.0, upright=True)
    for f in range(2):
        o_pts, o_desc, nc = orc.detect(op, frames[f], w, h, max_pts=8192)
        compare_frame(res["pts"][f], res["desc"][f], o_pts, o_desc, True)


def test_config5_4k_rotated_extended(surf, orc):
    """Config #5 layout: 3840x2160, 5 octaves, upright=false, 128-D, as an
    8-frame batch (XCD mapping, 4K integral near the int32 limit)."""
    w, h = 3840, 2160
    frames = surf.synth_frames(8, w, h, first=500)
    param = surf.make_param(5, 4.0, upright=False, extend=True)
    res = gpu_run(surf, param, frames, w, h, max_pts=32768)
    assert not res["truncated"]
    op = orc.make_param(5, 4.0, upright=False, extend=True)
    for f in (0, 7):
        o_pts, o_desc, nc = orc.detect(op, frames[f], w, h, max_pts=32768)
        assert len(o_pts) > 5000 and set(np.unique(o_pts["o"])) == {0, 1, 2, 3, 4}
        assert res["cand"][f] == nc
        compare_frame(res["pts"][f], res["desc"][f], o_pts, o_desc, False)


def _noise(n, w, h, seed):
    rng = np.random.default_rng(seed)
    pitch = (w + 127) // 128 * 128
    return rng.integers(0, 256, (n, h, pitch), dtype=np.uint8)


def test_sort_beyond_lds_capacity(surf, orc):
    """A noise frame at thresh 0.3 has ~21,700 keypoints: more than the
    16,384 candidates k_sort orders in LDS, so the global-scratch bitonic sort
    runs (candidate capacity 32,768)."""
    frames = _noise(1, W3, H3, 1)
    param = surf.make_param(4, 0.3, upright=False)
    res = gpu_run(surf, param, frames, W3, H3, max_pts=32768, cand_cap=32768)
    assert res["capacity"] == 32768 and not res["truncated"]
    op = orc.make_param(4, 0.3, upright=False)
    o_pts, o_desc, nc = orc.detect(op, frames[0], W3, H3, max_pts=32768)
    assert nc > 16384
    assert res["cand"][0] == nc
    compare_frame(res["pts"][0], res["desc"][0], o_pts, o_desc, False)


def test_candidate_capacity_truncation_is_deterministic(surf, orc):
    """More NMS survivors than the candidate capacity: the frame keeps the
    first `cap` survivors (scan order) -- the same set every run --, sorted
    canonically, each one a keypoint of the full result, and the detector
    reports the truncation (the reference keeps an arbitrary subset)."""
    frames = _noise(2, W3, H3, 2)
    param = surf.make_param(4, 0.3, upright=True)
    a = gpu_run(surf, param, frames, W3, H3, max_pts=32768, cand_cap=4096)
    b = gpu_run(surf, param, frames, W3, H3, max_pts=32768, cand_cap=4096)
    full = gpu_run(surf, param, frames, W3, H3, max_pts=32768, cand_cap=32768)
    assert a["truncated"] and b["truncated"] and not full["truncated"]
    for f in range(2):
        assert 0 < a["counts"][f] <= 4096
        assert a["pts"][f].tobytes() == b["pts"][f].tobytes()
        assert a["desc"][f].tobytes() == b["desc"][f].tobytes()
        key = lambda p: set(zip(p["o"].tolist(), p["y"].view(np.uint32).tolist(), p["x"].view(np.uint32).tolist(),
                                p["scale"].view(np.uint32).tolist()))
        assert key(a["pts"][f]) <= key(full["pts"][f])
        # canonical order: octave non-decreasing
        assert (np.diff(a["pts"][f]["o"]) >= 0).all()


@pytest.mark.parametrize("wsz,extend", [(2, False), (3, False), (5, False), (5, True), (6, True), (7, True)])
@pytest.mark.parametrize("upright", [True, False])
def test_descriptor_window_sizes(surf, orc, wsz, extend, upright):
    """desc_wsz other than 4 on the generic k_describe (surfd.cu:1566-1615,
    2391-2444 with wsz != 4): 16-, 36-, 100-, 200-, 288- and 392-D (mag_factor
    12 / wsz = 6, 4, 2, 2, 2, 1); windows past 4 x 4 x 8 use the 512-feature
    instance."""
    w, h = 640, 480
    frames = surf.synth_frames(2, w, h, first=40)
    param = surf.make_param(4, 4.0, upright=upright, extend=extend, desc_wsz=wsz)
    assert param.nfeatures == wsz * wsz * (8 if extend else 4)
    res = gpu_run(surf, param, frames, w, h)
    op = orc.make_param(4, 4.0, upright=upright, extend=extend, desc_wsz=wsz)
    for f in range(2):
        o_pts, o_desc, _ = orc.detect(op, frames[f], w, h)
        assert len(o_pts) > 100
        compare_frame(res["pts"][f], res["desc"][f], o_pts, o_desc, upright)


@pytest.mark.parametrize("case", ["doubled", "oct5", "oct6", "rotated_ext_720p"])
def test_gather_plan_cases(surf, orc, monkeypatch, case):
    """The single-frame plan (gather Hessian for every octave, the default
    for max_batch <= 8) on inputs the streaming tests cover: the doubled
    frame, 5 and 6 octaves, rotated 128-D."""
    monkeypatch.setenv("SURFHIP_HESS_GATHER", "1")
    doubled, noct, upright, extend, w, h = {
        "doubled": (True, 4, True, False, 640, 480),
        "oct5": (False, 5, True, False, 1920, 1080),
        "oct6": (False, 6, False, False, 1920, 1080),
        "rotated_ext_720p": (False, 5, False, True, 1280, 720),
    }[case]
    frames = surf.synth_frames(2, w, h, first=77)
    param = surf.make_param(noct, 4.0, doubled=doubled, upright=upright, extend=extend)
    res = gpu_run(surf, param, frames, w, h)
    op = orc.make_param(noct, 4.0, doubled=doubled, upright=upright, extend=extend)
    for f in range(2):
        o_pts, o_desc, _ = orc.detect(op, frames[f], w, h)
        assert len(o_pts) > 50
        compare_frame(res["pts"][f], res["desc"][f], o_pts, o_desc, upright)


@pytest.mark.parametrize("init_mask,doubled", [(15, True), (15, False), (12, False), (18, False), (6, False)])
def test_init_mask_sizes(surf, orc, init_mask, doubled):
    """Surfor::init's other initial lobes (surf.cpp:63-65: max_scale =
    init_mask_size / 3 + 2): lobe 5 (init_mask_size 15, 7 scales, 3 NMS levels)
    is main.cpp:195's setting for doubled images.  Planes bit-exact (the
    gather Hessian: the streaming kernels are compiled for lobe 3), keypoints
    bit-exact, descriptors within 1e-4 (halfImage from planes max_scale - 3 /
    max_scale - 1, NMS over levels k = 1, 3, .. < max_scale - 1)."""
    w, h = 640, 480
    frames = surf.synth_frames(2, w, h, first=90)
    param = surf.make_param(4, 2.0, doubled=doubled, init_mask_size=init_mask, upright=True)
    assert param.max_scale == init_mask // 3 + 2
    res = gpu_run(surf, param, frames, w, h, want_ws=True)
    op = orc.make_param(4, 2.0, doubled, init_mask, 2, True, False, 4)
    from test_gpu_parity import _plane_views
    for f in range(2):
        img = frames[f]
        _, ref, g, octs = orc.hessian(op, img, w, h)
        for (o, s, rp), (_, _, gp) in zip(_plane_views(ref, g, octs, op), _plane_views(res["resp"][f], g, octs, op)):
            same = rp.view(np.uint32) == gp.view(np.uint32)
            assert same.all(), f"octave {o} scale {s}: {(~same).sum()} cells differ"
        o_pts, o_desc, nc = orc.detect(op, img, w, h)
        assert len(o_pts) > 20
        assert res["cand"][f] == nc
        compare_frame(res["pts"][f], res["desc"][f], o_pts, o_desc, True)


def test_config5_per_rank_batch(surf, orc, monkeypatch):
    """Config #5 at the size one of its 8 ranks runs (bench.py): 64 frames of
    3840x2160, 5 octaves, rotated, 128-D, max_pts 262,144 -- frames 0, 7, 8,
    31, 63 against the oracle and all 64 against a single-frame detector (the
    gather plan: an independent Hessian path)."""
    w, h, n, max_pts, nf = 3840, 2160, 64, 262144, 128
    frames = surf.synth_frames(n, w, h, first=0)
    pitch = frames.shape[2]
    param = surf.make_param(5, 4.0, upright=False, extend=True)
    det = surf.Detector(param, w, h, max_batch=n, max_pts=max_pts)
    fb = surf.DeviceBuffer(frames.nbytes)
    fb.upload(frames)
    pb = surf.DeviceBuffer(48 * n * max_pts)
    db = surf.DeviceBuffer(4 * n * max_pts * nf)
    cb = surf.DeviceBuffer(4 * n)
    det.detect_batch(fb.ptr, n, pitch, h * pitch, pb.ptr, db.ptr, cb.ptr)
    surf.synchronize()
    counts = cb.download(np.int32, n)
    assert not det.truncated() and (counts < max_pts).all() and counts.min() > 5000
    cand = det.candidates(n)
    det.close()

    def frame_out(f):
        c = int(counts[f])
        pts = pb.download(surf.POINT_DTYPE, c, offset=48 * f * max_pts)
        d = db.download(np.float32, c * nf, offset=4 * f * max_pts * nf).reshape(c, nf)
        return pts, d

    op = orc.make_param(5, 4.0, upright=False, extend=True)
    for f in (0, 7, 8, 31, 63):
        o_pts, o_desc, nc = orc.detect(op, frames[f], w, h, max_pts=max_pts)
        assert cand[f] == nc
        pts, d = frame_out(f)
        compare_frame(pts, d, o_pts, o_desc, False)
    monkeypatch.delenv("SURFHIP_HESS_GATHER", raising=False)
    one = surf.Detector(param, w, h, max_batch=1, max_pts=max_pts)
    f1 = surf.DeviceBuffer(frames[0].nbytes)
    p1 = surf.DeviceBuffer(48 * max_pts)
    d1 = surf.DeviceBuffer(4 * max_pts * nf)
    c1 = surf.DeviceBuffer(4)
    for f in range(n):
        f1.upload(frames[f])
        one.detect_batch(f1.ptr, 1, pitch, 0, p1.ptr, d1.ptr, c1.ptr)
        surf.synchronize()
        c = int(c1.download(np.int32, 1)[0])
        assert c == counts[f], f
        pts, d = frame_out(f)
        assert_points_equal(p1.download(surf.POINT_DTYPE, c), pts)
        assert d1.download(np.float32, c * nf).tobytes() == d.tobytes(), f
    one.close()


@pytest.mark.parametrize("w,h,batch", [(5000, 360, 1), (8191, 200, 2)])
def test_wide_frames(surf, orc, w, h, batch):
    """Frames wider than 4,095 columns (the integral's 32-columns-per-thread
    path): integral and planes bit-exact, keypoints bit-exact, descriptors
    within 1e-4 (streaming Hessian kernels: conftest sets
    SURFHIP_HESS_GATHER=0)."""
    frames = surf.synth_frames(batch, w, h, first=300)
    param = surf.make_param(4, 4.0, upright=True)
    res = gpu_run(surf, param, frames, w, h, want_ws=True)
    op = orc.make_param(4, 4.0, upright=True)
    from test_gpu_parity import _plane_views
    for f in range(batch):
        ii_ref, ref, g, octs = orc.hessian(op, frames[f], w, h)
        ip = g.iwhp.z
        got_ii = res["ii"][f][: (h + 1) * ip].reshape(h + 1, ip)[:, : w + 1]
        assert np.array_equal(got_ii, ii_ref.reshape(h + 1, ip)[:, : w + 1])
        for (o, s, rp), (_, _, gp) in zip(_plane_views(ref, g, octs, op), _plane_views(res["resp"][f], g, octs, op)):
            same = rp.view(np.uint32) == gp.view(np.uint32)
            assert same.all(), f"octave {o} scale {s}: {(~same).sum()} cells differ"
        o_pts, o_desc, nc = orc.detect(op, frames[f], w, h)
        assert len(o_pts) > 100
        compare_frame(res["pts"][f], res["desc"][f], o_pts, o_desc, True)


def test_wide_frame_tight_pitch(surf, orc):
    """a wide frame (integral's 32-columns-per-thread path) with
    the smallest legal pitch, align16(W) with W % 32 in (0, 16]: the last
    16-byte half of a lane's 32 columns lies past the row (past the buffer on
    the last row) and must not be read.  The frames sit at the very end of a
    tight device buffer; integral bit-exact against the oracle."""
    w, h, n = 5000, 96, 2
    pitch = (w + 15) & ~15                     # 5008: 5000 % 32 = 8
    assert pitch % 32 == 16
    frames = surf.synth_frames(n, w, h, pitch=pitch, first=41)
    param = surf.make_param(4, 4.0, upright=True)
    det = surf.Detector(param, w, h, max_batch=n, max_pts=1024)
    fb = surf.DeviceBuffer(frames.nbytes)
    fb.upload(frames)
    det.run_integral(fb.ptr, n, pitch, h * pitch)
    surf.synchronize()
    ii, iis, _, _ = det.workspace()
    got = surf.download_ptr(ii, np.int32, n * iis).reshape(n, -1)
    for f in range(n):
        ii_ref = orc.integral(frames[f], w, h)
        ip = ii_ref.shape[1]
        assert np.array_equal(got[f][: (h + 1) * ip].reshape(h + 1, ip)[:, : w + 1], ii_ref[:, : w + 1]), f
    det.close()


def test_detector_rejects_oversized_grids(surf):
    """octave-0 sample grids past the NMS record fields (14-bit
    row / column, 13-bit block row) are rejected at creation instead of
    silently corrupting the candidate order."""
    param = surf.make_param(4, 4.0, upright=True, sampling_step=1)
    with pytest.raises(surf.SurfError):
        surf.Detector(param, 64, 16400, max_batch=1, max_pts=64)
    ok = surf.Detector(param, 64, 4000, max_batch=1, max_pts=64)
    ok.close()


def test_run_hessian_without_integral(surf):
    """run_hessian before any run_integral is an argument error
    (the u8 Hessian kernels would have no frames), not a HIP error."""
    param = surf.make_param(4, 4.0, upright=True)
    det = surf.Detector(param, 1920, 1080, max_batch=16, max_pts=1024)
    with pytest.raises(surf.SurfError, match="invalid argument"):
        det.run_hessian(16)
    det.close()


@pytest.mark.parametrize("fuse", ["1", "2"])
@pytest.mark.parametrize("w,h", [(960, 130), (1001, 97), (1002, 64), (1003, 71), (481, 50), (1025, 40),
                                 (1920, 1080)])
def test_fused_integral_from_hessian(surf, orc, monkeypatch, fuse, w, h):
    """plan.iiw: a u8 Hessian kernel's producers write the integral image
    (their strip integral plus k_ii_rowseg's row sums left of the strip), no
    separate integral pass -- k_hess_w (480-column strips, SURFHIP_II_FUSE=1)
    or k_hess_p0 (128-column strips, =2).  Bit-exact against the oracle for
    widths on and off both strip grids and every W % 4 (the lane holding
    column W stores only columns <= W; the pad columns stay 0), through
    detect_batch and through the pipelined entry point (row sums prefetched
    by the previous call)."""
    monkeypatch.setenv("SURFHIP_II_FUSE", fuse)
    n = 3
    frames = surf.synth_frames(n, w, h, first=900)
    pitch = frames.shape[2]
    param = surf.make_param(4, 4.0, upright=True)
    det = surf.Detector(param, w, h, max_batch=n, max_pts=4096)
    assert "writing the integral image" in det.hessian_kernels()
    assert ("(k_hess_p0)" in det.hessian_kernels()) == (fuse == "2")
    fb = [surf.DeviceBuffer(frames.nbytes) for _ in range(2)]
    fb[0].upload(frames)
    fb[1].upload(frames[::-1].copy())
    pb = surf.DeviceBuffer(48 * n * 4096)
    cb = surf.DeviceBuffer(4 * n)
    ip = surf.align_up(w + 1, 128)

    def check(order):
        surf.synchronize()
        ii, iis, _, _ = det.workspace()
        got = surf.download_ptr(ii, np.int32, n * iis).reshape(n, -1)
        for f in range(n):
            ref = orc.integral(frames[order[f]], w, h)
            assert np.array_equal(got[f][: (h + 1) * ip].reshape(h + 1, ip), ref), (w, h, f)

    det.detect_batch(fb[0].ptr, n, pitch, h * pitch, pb.ptr, None, cb.ptr)
    check([0, 1, 2])
    det.detect_batch_next(fb[1].ptr, n, pitch, h * pitch, pb.ptr, None, cb.ptr, fb[0].ptr, n, pitch, h * pitch)
    check([2, 1, 0])
    det.detect_batch_next(fb[0].ptr, n, pitch, h * pitch, pb.ptr, None, cb.ptr, None, 0, 0, 0)
    check([0, 1, 2])
    det.close()


@pytest.mark.parametrize("fuse", ["1", "2"])
def test_fused_integral_batch256(surf, orc, monkeypatch, fuse):
    """The fused integral of a full 256 x 1080p batch, frames spread over the
    batch, bit-exact against the oracle.  (k_hess_p0's integral stores with
    the row offset as the scalar offset left wrong values in rows 11-90 of
    every frame from 16 on, tools/ii_batch_check.py; 3-frame batches did not
    show it.)"""
    monkeypatch.setenv("SURFHIP_II_FUSE", fuse)
    n, w, h = 256, 1920, 1080
    frames = surf.synth_frames(n, w, h)
    pitch = frames.shape[2]
    param = surf.make_param(4, 4.0, upright=True)
    det = surf.Detector(param, w, h, max_batch=n, max_pts=8192)
    fb = surf.DeviceBuffer(frames.nbytes)
    fb.upload(frames)
    pb = surf.DeviceBuffer(48 * n * 8192)
    cb = surf.DeviceBuffer(4 * n)
    det.detect_batch(fb.ptr, n, pitch, h * pitch, pb.ptr, None, cb.ptr)
    surf.synchronize()
    ii, iis, _, _ = det.workspace()
    ip = surf.align_up(w + 1, 128)
    for f in [0, 1, 7, 8, 14, 15] + list(range(115, 136)) + [240, 255]:
        got = surf.download_ptr(ii + 4 * f * iis, np.int32, (h + 1) * ip).reshape(h + 1, ip)
        ref = orc.integral(frames[f], w, h)
        bad = np.argwhere(got != ref)
        assert len(bad) == 0, (fuse, f, len(bad), bad[:4].tolist())
    det.close()


def _fused_ii_with_guard(surf, frames, w, h, param, monkeypatch, fuse):
    """detect_batch of `frames` on a detector with one spare frame slot whose
    integral region holds a canary; returns (integral of every frame, the
    guard region after the last one, the canary)."""
    monkeypatch.setenv("SURFHIP_II_FUSE", fuse)
    n = len(frames)
    pitch = frames.shape[2]
    det = surf.Detector(param, w, h, max_batch=n + 1, max_pts=4096)
    assert "writing the integral image" in det.hessian_kernels()
    ii, iis, _, _ = det.workspace()
    canary = np.full(iis, 0x5A5A5A5A, np.uint32)
    surf.upload_ptr(ii + 4 * n * iis, canary)
    fb = surf.DeviceBuffer(frames.nbytes)
    fb.upload(frames)
    pb = surf.DeviceBuffer(48 * n * 4096)
    cb = surf.DeviceBuffer(4 * n)
    det.detect_batch(fb.ptr, n, pitch, h * pitch, pb.ptr, None, cb.ptr)
    surf.synchronize()
    got = surf.download_ptr(ii, np.int32, (n + 1) * iis).reshape(n + 1, iis)
    det.close()
    return got[:n], got[n].view(np.uint32), canary


@pytest.mark.parametrize("fuse", ["1", "2"])
@pytest.mark.parametrize("w,h", [(640, 240), (1920, 1040)])
def test_fused_integral_rows_past_frame_canary(surf, orc, monkeypatch, fuse, w, h):
    """VERDICT r05 item 1.  k_hess_w's producers walk 4 hw_nblk integral rows
    (hw_nblk: whole 20-block ring iterations), k_hess_p0's from row -16: for H
    = 80 m that is 79 rows past the frame's H + 1 -- the most any height gives.
    Frames' integrals are packed back to back (ii_stride = (H + 1) ip), so a
    store of those rows that the range check let through would land in the
    next frame's first rows or, after the last frame, in the spare slot's
    canary.  Every frame bit-exact, the canary intact."""
    hw_nblk = ((h // 4 + 1 + 19) // 20) * 20
    assert 4 * hw_nblk - (h + 1) == 79
    n = 16
    frames = surf.synth_frames(n, w, h, first=4000)
    param = surf.make_param(4, 4.0, upright=True)
    got, guard, canary = _fused_ii_with_guard(surf, frames, w, h, param, monkeypatch, fuse)
    ip = surf.align_up(w + 1, 128)
    for f in range(n):
        ref = orc.integral(frames[f], w, h)
        bad = np.argwhere(got[f][: (h + 1) * ip].reshape(h + 1, ip) != ref)
        assert len(bad) == 0, (fuse, f, len(bad), bad[:4].tolist())
    assert np.array_equal(guard, canary), (fuse, int((guard != canary).sum()))


@pytest.mark.parametrize("fuse", ["1", "2"])
def test_fused_integral_saturated_4k(surf, orc, monkeypatch, fuse):
    """the all-255 3840 x 2160 frame through the fused
    writers (k_hess_w's / k_hess_p0's producers, 5 octaves as config #5): the
    image's integral tops out at 2,115,072,000 (< 2^31) and the producers'
    uint32 carries must reach it exactly; canary after the frame intact."""
    w, h = 3840, 2160
    frames = np.full((1, h, surf.align_up(w, 128)), 255, np.uint8)
    param = surf.make_param(5, 4.0, upright=True)
    got, guard, canary = _fused_ii_with_guard(surf, frames, w, h, param, monkeypatch, fuse)
    ip = surf.align_up(w + 1, 128)
    ii0 = got[0][: (h + 1) * ip].reshape(h + 1, ip)
    assert ii0[h, w] == 255 * w * h
    np.testing.assert_array_equal(ii0, orc.integral(frames[0], w, h))
    assert np.array_equal(guard, canary)


def test_fused_integral_switch(surf, monkeypatch):
    """SURFHIP_II_FUSE=0 keeps the separate integral passes (A/B); the gather
    plan (few frames) never fuses; a 5-octave plan does (octave 4's k_hessian
    reads the integral k_hess_w wrote, after it on the same stream)."""
    param = surf.make_param(4, 4.0, upright=True)
    monkeypatch.setenv("SURFHIP_II_FUSE", "0")
    det = surf.Detector(param, 640, 480, max_batch=16, max_pts=1024)
    assert "integral" not in det.hessian_kernels()
    det.close()
    monkeypatch.delenv("SURFHIP_II_FUSE")
    monkeypatch.setenv("SURFHIP_HESS_GATHER", "1")
    det = surf.Detector(param, 640, 480, max_batch=16, max_pts=1024)
    assert "integral" not in det.hessian_kernels()
    det.close()
    monkeypatch.setenv("SURFHIP_HESS_GATHER", "0")
    det = surf.Detector(surf.make_param(5, 4.0, upright=True), 1920, 1080, max_batch=16, max_pts=1024)
    assert "writing the integral image" in det.hessian_kernels() and "k_hessian (octave 4)" in det.hessian_kernels()
    det.close()
