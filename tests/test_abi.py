"""CPU tests of the boundary (no GPU, no compute calls): the C-ABI library
loads and exports every entry point include/surfhip.h declares, the C++
drop-in library exports the surf.h API, parameter derivation matches the
oracle, main.cpp-style callers compile against include/, and the
multi-GPU slab format round-trips."""
from __future__ import annotations

import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO

INC = os.path.join(REPO, "include")
PKG = os.path.join(REPO, "cuda-surf_amd")


def declared_functions(header: str):
    src = open(os.path.join(INC, header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(surfhip_[a-z0-9_]+)\s*\(", src)))


def exported(lib: str, demangle=False):
    out = subprocess.check_output(["nm", "-D", "--defined-only"] + (["-C"] if demangle else []) + [lib], text=True)
    return out


def test_surfhip_exports_every_declared_symbol(surf):
    names = declared_functions("surfhip.h")
    assert len(names) >= 40
    syms = exported(os.path.join(PKG, "libsurfhip.so"))
    missing = [n for n in names if not re.search(rf"\bT {n}$", syms, flags=re.M)]
    assert not missing, missing
    for n in names:                       # and ctypes resolves each one
        getattr(surf.lib, n)


def test_surfcomm_exports_every_declared_symbol():
    """libsurfcomm.so (RCCL exchange of packed slabs, include/surfhip_comm.h)
    exports every declared entry point; no GPU call is made."""
    lib = os.path.join(PKG, "libsurfcomm.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-C", PKG, "libsurfcomm.so"])
    names = declared_functions("surfhip_comm.h")
    assert len(names) >= 6
    syms = exported(lib)
    missing = [n for n in names if not re.search(rf"\bT {n}$", syms, flags=re.M)]
    assert not missing, missing


def test_libsurf_exports_reference_api():
    lib = os.path.join(PKG, "libsurf.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-C", PKG, "libsurf.so"])
    syms = exported(lib, demangle=True)
    for sig in ("surf::initSurfData(surf::SurfData&, int, bool, bool)",
                "surf::freeSurfData(surf::SurfData&)",
                "surf::Surfor::Surfor()", "surf::Surfor::~Surfor()",
                "surf::Surfor::init(int, float, bool, int, int, bool, bool, int, int, int)",
                "surf::Surfor::detectAndCompute(unsigned char*, surf::SurfData&, int3, float**, bool)",
                "surf::Surfor::match(surf::SurfData&, surf::SurfData&, float*, float*)"):
        assert sig in syms, sig


def test_make_param_matches_oracle(surf, orc):
    for noct in (1, 4, 5, 8):
        for upright in (False, True):
            for extend in (False, True):
                for wsz in (1, 2, 3, 4, 5, 6, 7, 8, 12):
                    for dbl in (False, True):
                        nf = wsz * wsz * (8 if extend else 4)
                        if wsz > 7:                    # the reference reads past lookup2[40]
                            with pytest.raises(surf.SurfError):
                                surf.make_param(noct, 4.0, dbl, 9, 2, upright, extend, wsz)
                            with pytest.raises(ValueError):
                                orc.make_param(noct, 4.0, dbl, 9, 2, upright, extend, wsz)
                            continue
                        b = orc.make_param(noct, 4.0, dbl, 9, 2, upright, extend, wsz)
                        a = surf.make_param(noct, 4.0, dbl, 9, 2, upright, extend, wsz)
                        assert bytes(a) == bytes(b)
                        assert a.mag_factor == 12 // wsz and a.nfeatures == nf    # surf.cpp:77-79


def test_make_param_rejects_out_of_scope(surf):
    with pytest.raises(surf.SurfError):
        surf.make_param(4, 4.0, init_mask_size=21)     # max_scale 9 > MAX_SCALE (surfd.h:9)
    with pytest.raises(surf.SurfError):
        surf.make_param(4, 4.0, init_mask_size=5)      # max_scale 3: degenerate lobes
    with pytest.raises(surf.SurfError):
        surf.make_param(0, 4.0)
    with pytest.raises(surf.SurfError):
        surf.make_param(4, 4.0, desc_wsz=8)             # weights past lookup2[40] (surfd.cu:23)


@pytest.mark.parametrize("init_mask", [6, 9, 12, 15, 18, 20])
def test_make_param_init_mask_sizes_match_oracle(surf, orc, init_mask):
    """Surfor::init with the reference's other initial lobes (main.cpp:195:
    lobe 5 = init_mask_size 15 for doubled images): max_scale = lobe + 2,
    4 .. MAX_SCALE."""
    for dbl in (False, True):
        a = surf.make_param(4, 4.0, dbl, init_mask, 2, True, False, 4)
        b = orc.make_param(4, 4.0, dbl, init_mask, 2, True, False, 4)
        assert bytes(a) == bytes(b) and a.max_scale == init_mask // 3 + 2


def test_errors_without_gpu_are_reported(surf):
    """The product path fails loudly (no CPU fallback) when no GPU is present."""
    if surf.device_count.__doc__ is None:
        pass
    try:
        n = surf.device_count()
    except surf.SurfError:
        return                                          # expected in the build container
    assert n >= 1


def test_drop_in_headers_compile():
    """A main.cpp-shaped caller (tools/surf_demo.cpp) compiles and links
    against include/ + libsurf.so exactly as the reference's main.cpp uses
    surf.h and cuda_utils.h."""
    out = os.path.join("/tmp", "surf_demo_test")
    subprocess.check_call(["make", "-s", "-C", PKG, "libsurf.so"])
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-I", INC, os.path.join(REPO, "tools", "surf_demo.cpp"),
                           "-L", PKG, "-lsurf", "-lsurfhip", "-lsurfsynth", f"-Wl,-rpath,{PKG}", "-o", out])
    assert os.path.exists(out)


def test_struct_offsets_in_headers():
    """surf_structures.h static_asserts the reference layout; compile it."""
    src = '#include "surf_structures.h"\nint main(){return sizeof(surf::SurfPoint)+sizeof(surf::SurfParam);}\n'
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", INC, "-x", "c++", "-"], input=src, text=True,
                   check=True)


def test_slab_roundtrip(surf):
    rng = np.random.default_rng(7)
    counts = rng.integers(0, 50, 5).astype(np.int32)
    total = int(counts.sum())
    pts = np.zeros(total, surf.POINT_DTYPE)
    pts["x"] = rng.random(total)
    pts["o"] = rng.integers(0, 4, total)
    desc = rng.random((total, 64)).astype(np.float32)
    buf = surf.build_slab(counts, pts, desc)
    assert len(buf) == surf.lib.surfhip_slab_bytes(5, total, 64)
    c2, p2, d2 = surf.parse_slab(buf)
    np.testing.assert_array_equal(c2, counts)
    assert p2.tobytes() == pts.tobytes()
    np.testing.assert_array_equal(d2, desc)


def test_shard_ranges(surf):
    for n, world in ((2048, 8), (512, 8), (10, 3), (1, 2)):
        spans = [surf.dist.shard_range(n, world, r) for r in range(world)]
        assert spans[0][0] == 0
        assert sum(c for _, c in spans) == n
        for (s0, c0), (s1, _) in zip(spans, spans[1:]):
            assert s0 + c0 == s1


def test_dump_file_roundtrip(surf, tmp_path):
    """Keypoint file (surfhip_dump_append, host-only C): records of slabs
    with and without descriptors read back byte-for-byte; bad input and a
    truncated file are rejected."""
    rng = np.random.default_rng(11)
    path = str(tmp_path / "kp.surfkpd")
    param = surf.make_param(4, 4.0, False, 9, 2, True, False, 4)
    recs = []
    for i, (nframes, nf) in enumerate(((3, 64), (1, 0), (4, 128), (2, 64))):
        counts = rng.integers(0, 40, nframes).astype(np.int32)
        counts[0] = 0                                           # an empty frame
        total = int(counts.sum())
        pts = np.zeros(total, surf.POINT_DTYPE)
        pts["x"], pts["y"] = rng.random(total) * 1920, rng.random(total) * 1080
        pts["laplace"] = rng.integers(0, 2, total)
        desc = rng.random((total, nf)).astype(np.float32) if nf else None
        slab = surf.build_slab(counts, pts, desc)
        surf.dump_append(path, slab, 1920, 1080, param, first_frame=100 * i)
        recs.append((counts, pts, desc))
    back = surf.read_dump(path)
    assert len(back) == len(recs)
    for i, ((hdr, c, p, d), (c0, p0, d0)) in enumerate(zip(back, recs)):
        assert hdr["magic"] == b"SURFKPD1" and hdr["width"] == 1920 and hdr["height"] == 1080
        assert hdr["first_frame"] == 100 * i and hdr["upright"] == 1 and hdr["noctaves"] == 4
        assert hdr["thresh"] == np.float32(4.0)
        np.testing.assert_array_equal(c, c0)
        assert p.tobytes() == p0.tobytes()
        if d0 is None:
            assert d is None and hdr["nfeatures"] == 0
        else:
            assert d.tobytes() == d0.tobytes()
    good = surf.build_slab(np.array([2], np.int32), np.zeros(2, surf.POINT_DTYPE), None)
    with pytest.raises(surf.SurfError):                          # slab size disagrees with its header
        surf.dump_append(path, good[:-4], 64, 48, param)
    raw = open(path, "rb").read()
    bad = str(tmp_path / "trunc.surfkpd")
    open(bad, "wb").write(raw[:-10])
    with pytest.raises(ValueError):
        surf.read_dump(bad)
