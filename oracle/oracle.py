"""ctypes binding of the CPU oracle (liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product path.  Parity status of
the oracle itself: "parity unpinned" vs the CUDA reference binary (see
surf_oracle.h and DESIGN.md).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

POINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("scale", "<f4"), ("o", "<i4"),
                        ("strength", "<f4"), ("laplace", "<i4"), ("ori", "<f4"),
                        ("score", "<f4"), ("match", "<i4"), ("match_x", "<f4"),
                        ("match_y", "<f4"), ("ambiguity", "<f4")])


class Param(C.Structure):
    _fields_ = [("thresh", C.c_float), ("init_lobe", C.c_int), ("doubled", C.c_bool),
                ("max_scale", C.c_int), ("noctaves", C.c_int), ("sampling", C.c_int),
                ("divisor", C.c_float), ("upright", C.c_bool), ("extend", C.c_bool),
                ("desc_wsz", C.c_int), ("mag_factor", C.c_int), ("orient_size", C.c_int),
                ("nfeatures", C.c_int)]


class Int3(C.Structure):
    _fields_ = [("x", C.c_int), ("y", C.c_int), ("z", C.c_int)]


class Geom(C.Structure):
    _fields_ = [("iwhp", Int3), ("swhp", Int3 * 8), ("osize", C.c_int * 8),
                ("ooff", C.c_size_t * 8), ("tot_osize", C.c_size_t)]


class Octave(C.Structure):
    _fields_ = [("octave", C.c_int), ("init_scale", C.c_int), ("nscale", C.c_int), ("delta", C.c_int),
                ("mask", C.c_int * 8), ("border1", C.c_int * 8), ("x2", C.c_int * 8),
                ("x3", C.c_int * 8), ("x4", C.c_int * 8), ("norm", C.c_float * 8),
                ("borders", C.c_int * 8), ("mborders", C.c_int * 3), ("nms_gx", C.c_int),
                ("nms_gy", C.c_int)]


def ensure_built() -> None:
    src = os.path.join(HERE, "surf_oracle.c")
    newest = max(os.path.getmtime(src), os.path.getmtime(os.path.join(HERE, "surf_oracle.h")))
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        subprocess.check_call(["make", "-s", "-C", HERE])


ensure_built()
_L = C.CDLL(LIB)
_vp, _i = C.c_void_p, C.c_int
_L.or_init_param.restype = _i
_L.or_init_param.argtypes = [C.POINTER(Param), _i, C.c_float, C.c_bool, _i, _i, C.c_bool, C.c_bool, _i]
_L.or_init_tables.argtypes = [_vp, _vp, _vp]
_L.or_geometry.argtypes = [C.POINTER(Param), _i, _i, C.POINTER(Geom)]
_L.or_octave_params.argtypes = [C.POINTER(Param), C.POINTER(Geom), C.POINTER(Octave)]
_L.or_integral.argtypes = [_vp, _i, _i, _i, _vp, _i]
_L.or_hessian.argtypes = [C.POINTER(Param), C.POINTER(Geom), C.POINTER(Octave), _vp, _vp]
_L.or_find_points.restype = _i
_L.or_find_points.argtypes = [C.POINTER(Param), C.POINTER(Geom), C.POINTER(Octave), _vp, _vp, _vp, _i]
_L.or_detect_and_compute.restype = _i
_L.or_detect_and_compute.argtypes = [C.POINTER(Param), _vp, _i, _i, _i, _vp, _i, _vp, C.POINTER(_i)]
_L.or_sinf.restype = C.c_float
_L.or_sinf.argtypes = [C.c_float]
_L.or_cosf.restype = C.c_float
_L.or_cosf.argtypes = [C.c_float]
_L.or_fast_atan2.restype = C.c_float
_L.or_fast_atan2.argtypes = [C.c_float, C.c_float]
_L.or_bench_frames.restype = C.c_double
_L.or_bench_frames.argtypes = [C.POINTER(Param), _vp, _i, _i, _i, _i, C.c_size_t, _i, _i,
                               C.POINTER(C.c_longlong)]
_L.or_test_solve3.argtypes = [_vp, _vp]
_L.or_test_fit.restype = C.c_float
_L.or_test_fit.argtypes = [_vp, _vp, _i, _i, _i, _i, _i]
_L.or_test_box.restype = C.c_uint32
_L.or_test_box.argtypes = [_vp, _i, _i, _i, _i, _i]
_L.or_test_place.argtypes = [_vp, _i, _i, C.c_float, _i, C.c_float, _i, C.c_float, C.c_float]

_L.or_double_image.argtypes = [_vp, _i, _i, _i, _vp, _i]
_L.or_orientation.restype = C.c_float
_L.or_orientation.argtypes = [C.POINTER(Param), C.POINTER(Geom), _vp, _vp, _vp, _vp]
_L.or_describe.argtypes = [C.POINTER(Param), C.POINTER(Geom), _vp, _vp, _vp, _vp]
_L.or_match.argtypes = [_vp, _vp, _vp, _vp, _i, _i, _i, _i]

lib = _L


def make_param(noctaves=4, thresh=0.2, doubled=False, init_mask_size=9, sampling_step=2,
               upright=False, extend=False, desc_wsz=4) -> Param:
    p = Param()
    rc = _L.or_init_param(C.byref(p), noctaves, thresh, doubled, init_mask_size, sampling_step,
                          upright, extend, desc_wsz)
    if rc != 0:
        raise ValueError("unsupported oracle parameters")
    return p


def tables():
    l1 = np.zeros(83, np.float32)
    l2 = np.zeros(40, np.float32)
    b = np.zeros(72, np.float32)
    _L.or_init_tables(l1.ctypes.data, l2.ctypes.data, b.ctypes.data)
    return l1, l2, b


def geometry(p: Param, w: int, h: int):
    g = Geom()
    _L.or_geometry(C.byref(p), w, h, C.byref(g))
    octs = (Octave * 8)()
    _L.or_octave_params(C.byref(p), C.byref(g), octs)
    return g, octs


def integral(img: np.ndarray, w: int, h: int) -> np.ndarray:
    """(H+1) x align128(W+1) int32, as the reference lays it out."""
    img = np.ascontiguousarray(img)
    ip = (w + 1 + 127) // 128 * 128
    ii = np.zeros((h + 1, ip), np.int32)
    _L.or_integral(img.ctypes.data, w, h, img.shape[1], ii.ctypes.data, ip)
    return ii


def double_image(img: np.ndarray, w: int, h: int) -> np.ndarray:
    """The doubled image D (2h-2 rows x 2w-2 columns, u8) of cuIntegralDoubleU4."""
    img = np.ascontiguousarray(img)
    out = np.zeros((2 * h - 2, 2 * w - 2), np.uint8)
    _L.or_double_image(img.ctypes.data, w, h, img.shape[1], out.ctypes.data, out.shape[1])
    return out


def describe_points(p: Param, g: Geom, ii: np.ndarray, pts: np.ndarray, orient: bool = True):
    """or_orientation (rotated) + or_describe of given points on an integral
    image: (ori[n], desc[n, nf]); the points' own ori is used when
    orient is False."""
    l1, l2, bins = tables()
    ii = np.ascontiguousarray(ii, np.int32)
    pts = np.ascontiguousarray(pts, dtype=POINT_DTYPE).copy()
    desc = np.zeros((len(pts), p.nfeatures), np.float32)
    for i in range(len(pts)):
        pp = pts[i:i + 1]
        if not p.upright and orient:
            pts["ori"][i] = _L.or_orientation(C.byref(p), C.byref(g), ii.ctypes.data, l1.ctypes.data,
                                              bins.ctypes.data, pp.ctypes.data)
            pp = pts[i:i + 1]
        _L.or_describe(C.byref(p), C.byref(g), ii.ctypes.data, l2.ctypes.data, pp.ctypes.data,
                       desc[i].ctypes.data)
    return pts["ori"].copy(), desc


def hessian(p: Param, img: np.ndarray, w: int, h: int):
    """Integral image + all response planes (flat float array, reference layout)."""
    g, octs = geometry(p, w, h)
    if p.doubled:                                    # surf.cpp:234-235
        ii = integral(double_image(img, w, h), 2 * w - 2, 2 * h - 2)
    else:
        ii = integral(img, w, h)
    resp = np.zeros(g.tot_osize, np.float32)
    _L.or_hessian(C.byref(p), C.byref(g), octs, ii.ctypes.data, resp.ctypes.data)
    return ii, resp, g, octs


def detect(p: Param, img: np.ndarray, w: int, h: int, max_pts: int = 65536, desc: bool = True):
    """or_detect_and_compute: (points[n] structured, descriptors[n, nf] or None, n_candidates)."""
    img = np.ascontiguousarray(img)
    pts = np.zeros(max_pts, POINT_DTYPE)
    d = np.zeros((max_pts, p.nfeatures), np.float32) if desc else None
    nc = C.c_int()
    n = _L.or_detect_and_compute(C.byref(p), img.ctypes.data, w, h, img.shape[1], pts.ctypes.data,
                                 max_pts, d.ctypes.data if desc else None, C.byref(nc))
    if n < 0:
        raise RuntimeError("oracle detect failed")
    return pts[:n].copy(), (d[:n].copy() if desc else None), nc.value


def bench_frames(p: Param, frames: np.ndarray, w: int, h: int, max_pts: int, nthreads: int):
    frames = np.ascontiguousarray(frames)
    tot = C.c_longlong()
    secs = _L.or_bench_frames(C.byref(p), frames.ctypes.data, frames.shape[0], w, h, frames.shape[2],
                              frames.shape[1] * frames.shape[2], max_pts, nthreads, C.byref(tot))
    return secs, tot.value


def match(pts1: np.ndarray, pts2: np.ndarray, f1: np.ndarray, f2: np.ndarray,
          full_tail: bool = False) -> np.ndarray:
    """or_match (findMaxCorr restated): a copy of pts1 with score, match,
    match_x, match_y, ambiguity filled in."""
    out = np.ascontiguousarray(pts1, dtype=POINT_DTYPE).copy()
    pts2 = np.ascontiguousarray(pts2, dtype=POINT_DTYPE)
    f1 = np.ascontiguousarray(f1, dtype=np.float32)
    f2 = np.ascontiguousarray(f2, dtype=np.float32)
    n1, n2 = len(out), len(pts2)
    nf = f1.shape[1] if f1.ndim == 2 else (f2.shape[1] if f2.ndim == 2 else 64)
    assert f1.shape == (n1, nf) and f2.shape == (n2, nf)
    _L.or_match(out.ctypes.data, pts2.ctypes.data, f1.ctypes.data, f2.ctypes.data,
                n1, n2, nf, int(bool(full_tail)))
    return out


REF_LIB = os.path.join(HERE, "_ref", "libref_host.so")


def ref_host():
    """The reference's own host C++ (oracle/ref_extract.py), or None where
    /root/reference was not there to build it from."""
    if not os.path.exists(REF_LIB):
        return None
    L = C.CDLL(REF_LIB)
    L.ref_solve.argtypes = [_vp, _vp]
    L.ref_fit.restype = C.c_float
    L.ref_fit.argtypes = [_vp, _vp, _i, _i, _i, _i, _i]
    L.ref_hessian_params.argtypes = [_i, _i, _i, _i, C.POINTER(_i), _i, _vp, _i, _i, _vp, _vp]
    L.ref_init_lut.argtypes = [_vp, _vp]
    L.ref_octave_plan.argtypes = [_i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp]
    L.ref_surfor_init.argtypes = [_vp, _i, C.c_float, _i, _i, _i, _i, _i, _i, _i, _i]
    L.ref_alloc_geometry.restype = _i
    L.ref_alloc_geometry.argtypes = [_i, _i, _i, _i, _i, _i, _vp, _vp, _vp]
    L.ref_nms_grid.argtypes = [_i, _vp, _i, _i, _vp, _vp]
    return L
