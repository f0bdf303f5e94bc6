"""surf_amd -- Python host-side mirror of the CUDA-SURF interface on MI355X.

The compute path is the in-tree HIP library ``libsurfhip.so`` (C-ABI,
``include/surfhip.h``); this module only binds it with ctypes and mirrors the
reference host API (``surf.h``: ``Surfor.init`` / ``Surfor.detectAndCompute``,
``initSurfData`` / ``freeSurfData``) so tests and the bench read like the
reference's own usage in ``main.cpp:163-283``.

There is no CPU fallback: if ``libsurfhip.so`` is missing or fails to load,
importing this package raises.  (The CPU oracle under ``oracle/`` is test
infrastructure and is never imported from here.)

The directory name ``cuda-surf_amd`` is not a valid identifier, so callers
load it with :func:`load_package` semantics (see ``tests/conftest.py``)::

    spec = importlib.util.spec_from_file_location("surf_amd", ".../cuda-surf_amd/__init__.py")
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(_HERE)

# ----------------------------------------------------------------- layouts
# surf_structures.h:10-30 (48 B) and :45-72 (48 B), byte-identical.


class SurfPoint(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("scale", C.c_float), ("o", C.c_int),
                ("strength", C.c_float), ("laplace", C.c_int), ("ori", C.c_float),
                ("score", C.c_float), ("match", C.c_int), ("match_x", C.c_float),
                ("match_y", C.c_float), ("ambiguity", C.c_float)]


class SurfParam(C.Structure):
    _fields_ = [("thresh", C.c_float), ("init_lobe", C.c_int), ("doubled", C.c_bool),
                ("max_scale", C.c_int), ("noctaves", C.c_int), ("sampling", C.c_int),
                ("divisor", C.c_float), ("upright", C.c_bool), ("extend", C.c_bool),
                ("desc_wsz", C.c_int), ("mag_factor", C.c_int), ("orient_size", C.c_int),
                ("nfeatures", C.c_int)]


assert C.sizeof(SurfPoint) == 48 and C.sizeof(SurfParam) == 48

POINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("scale", "<f4"), ("o", "<i4"),
                        ("strength", "<f4"), ("laplace", "<i4"), ("ori", "<f4"),
                        ("score", "<f4"), ("match", "<i4"), ("match_x", "<f4"),
                        ("match_y", "<f4"), ("ambiguity", "<f4")])
assert POINT_DTYPE.itemsize == 48

H2H, H2D, D2H, D2D = 0, 1, 2, 3
NSTAGE = 6
STAGES = ("integral", "hessian", "nms", "sort", "describe", "total")

# ------------------------------------------------------------------ library

# SURFHIP_LIB_DIR: a directory holding an alternative build of libsurfhip.so
# (diagnostic kernel variants, tools/diag_build.sh); the default is in-tree.
LIB_PATH = os.path.join(os.environ.get("SURFHIP_LIB_DIR") or _HERE, "libsurfhip.so")
SYNTH_PATH = os.path.join(_HERE, "libsurfsynth.so")

# The HIP runtime must be a single copy per process: if PyTorch is already
# imported its bundled libamdhip64 (same soname) satisfies ours.
if not os.path.exists(LIB_PATH):
    raise ImportError(f"surf_amd: {LIB_PATH} is missing -- run `make -C cuda-surf_amd` "
                      "(or __graft_entry__.build()); there is no CPU fallback")
_lib = C.CDLL(LIB_PATH)
_syn = C.CDLL(SYNTH_PATH)

_vp, _i, _sz = C.c_void_p, C.c_int, C.c_size_t
_sigs = {
    "surfhip_error_string": (C.c_char_p, [_i]),
    "surfhip_last_hip_error": (_i, []),
    "surfhip_get_device_count": (_i, [C.POINTER(_i)]),
    "surfhip_set_device": (_i, [_i]),
    "surfhip_get_device": (_i, [C.POINTER(_i)]),
    "surfhip_device_name": (_i, [_i, C.c_char_p, _i, C.POINTER(_i)]),
    "surfhip_versions": (_i, [C.POINTER(_i), C.POINTER(_i)]),
    "surfhip_malloc": (_i, [C.POINTER(_vp), _sz]),
    "surfhip_malloc_pitch": (_i, [C.POINTER(_vp), C.POINTER(_sz), _sz, _sz]),
    "surfhip_free": (_i, [_vp]),
    "surfhip_memset": (_i, [_vp, _i, _sz]),
    "surfhip_memset_async": (_i, [_vp, _i, _sz, _vp]),
    "surfhip_memcpy": (_i, [_vp, _vp, _sz, _i]),
    "surfhip_memcpy_async": (_i, [_vp, _vp, _sz, _i, _vp]),
    "surfhip_memcpy2d": (_i, [_vp, _sz, _vp, _sz, _sz, _sz, _i]),
    "surfhip_device_synchronize": (_i, []),
    "surfhip_device_reset": (_i, []),
    "surfhip_stream_create": (_i, [C.POINTER(_vp)]),
    "surfhip_stream_destroy": (_i, [_vp]),
    "surfhip_stream_synchronize": (_i, [_vp]),
    "surfhip_event_create": (_i, [C.POINTER(_vp)]),
    "surfhip_event_destroy": (_i, [_vp]),
    "surfhip_event_record": (_i, [_vp, _vp]),
    "surfhip_event_synchronize": (_i, [_vp]),
    "surfhip_event_elapsed": (_i, [C.POINTER(C.c_float), _vp, _vp]),
    "surfhip_detector_create": (_i, [C.POINTER(_vp), C.POINTER(SurfParam), _i, _i, _i, _i, _i, _vp]),
    "surfhip_detector_destroy": (_i, [_vp]),
    "surfhip_detector_set_stream": (_i, [_vp, _vp]),
    "surfhip_make_param": (_i, [C.POINTER(SurfParam), _i, C.c_float, _i, _i, _i, _i, _i, _i]),
    "surfhip_detect_batch": (_i, [_vp, _vp, _i, _i, _sz, _vp, _vp, _vp]),
    "surfhip_detect_batch_next": (_i, [_vp, _vp, _i, _i, _sz, _vp, _vp, _vp, _vp, _i, _i, _sz]),
    "surfhip_detector_drain": (_i, [_vp]),
    "surfhip_detect": (_i, [_vp, _vp, _i, _vp, _i, C.POINTER(_i), C.POINTER(_vp), _i]),
    "surfhip_detector_candidates": (_i, [_vp, C.POINTER(_i), _i]),
    "surfhip_detector_status": (_i, [_vp, C.POINTER(_i)]),
    "surfhip_detector_capacity": (_i, [_vp, C.POINTER(_i)]),
    "surfhip_detector_set_profiling": (_i, [_vp, _i]),
    "surfhip_detector_stage_times": (_i, [_vp, C.POINTER(C.c_float)]),
    "surfhip_detector_time_hessian": (_i, [_vp, _i]),
    "surfhip_detector_hessian_times": (_i, [_vp, C.POINTER(C.c_float), _i, C.POINTER(_i)]),
    "surfhip_detector_workspace": (_i, [_vp, C.POINTER(_vp), C.POINTER(_sz), C.POINTER(_vp), C.POINTER(_sz)]),
    "surfhip_detector_geometry": (_i, [_vp, C.POINTER(_i), C.POINTER(_i), C.POINTER(C.c_longlong), C.POINTER(_i)]),
    "surfhip_run_integral": (_i, [_vp, _vp, _i, _i, _sz]),
    "surfhip_run_hessian": (_i, [_vp, _i]),
    "surfhip_hessian_bytes_per_frame": (C.c_longlong, [_vp]),
    "surfhip_hessian_plan": (C.c_int, [_vp, C.c_char_p, C.c_int]),
    "surfhip_slab_bytes": (_sz, [_i, _i, _i]),
    "surfhip_batch_total": (_i, [_vp, _i, C.POINTER(_i)]),
    "surfhip_pack_slab": (_i, [_vp, _vp, _vp, _vp, _i, _vp]),
    "surfhip_pack_slab_cap": (_i, [_vp, _vp, _vp, _vp, _i, _vp, _sz]),
    "surfhip_match_scratch": (_sz, [_i, _i, _i]),
    "surfhip_match": (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp]),
    "surfhip_ingest_create": (_i, [C.POINTER(_vp), _vp, _i]),
    "surfhip_ingest_destroy": (_i, [_vp]),
    "surfhip_ingest_acquire": (_i, [_vp, C.POINTER(_vp), C.POINTER(_i), C.POINTER(_sz)]),
    "surfhip_ingest_submit": (_i, [_vp, _i]),
    "surfhip_ingest_collect": (_i, [_vp, C.POINTER(_vp), C.POINTER(_sz)]),
    "surfhip_ingest_pending": (_i, [_vp, C.POINTER(_i)]),
    "surfhip_dump_append": (_i, [C.c_char_p, _vp, _sz, _i, _i, C.POINTER(SurfParam), C.c_longlong]),
    "surfhip_build_info": (C.c_char_p, []),
    "surfhip_stream_run": (_i, [_i, _vp, _vp, _sz, _vp]),
    "surfhip_stream_wait_event": (_i, [_vp, _vp]),
    "surfhip_detector_set_describe_event": (_i, [_vp, _vp]),
    "surfhip_stream_bytes": (_sz, [_i, _sz]),
}
for _name, (_res, _args) in _sigs.items():
    _f = getattr(_lib, _name)
    _f.restype = _res
    _f.argtypes = _args

_syn.surf_synth_frames.restype = _i
_syn.surf_synth_frames.argtypes = [_vp, _i, _i, _i, _i, _sz, _i, _i, _i]
_syn.surf_synth_default_blobs.restype = _i
_syn.surf_synth_default_blobs.argtypes = [_i, _i]
_syn.surf_pgm_info.restype = C.c_long
_syn.surf_pgm_info.argtypes = [C.c_char_p, C.POINTER(_i), C.POINTER(_i)]
_syn.surf_pgm_read.restype = _i
_syn.surf_pgm_read.argtypes = [C.c_char_p, _vp, _i]
_syn.surf_downsample2.restype = None
_syn.surf_downsample2.argtypes = [_vp, _i, _i, _i, _vp, _i]

lib = _lib


class SurfError(RuntimeError):
    pass


def check(rc: int, what: str = "") -> None:
    """CHECK() of cuda_utils.h:18-25, raising instead of exit(-1)."""
    if rc != 0:
        msg = _lib.surfhip_error_string(rc).decode()
        raise SurfError(f"{what}: {msg} (status {rc}, hip {_lib.surfhip_last_hip_error()})")


def build_info() -> str:
    return _lib.surfhip_build_info().decode()


def align_up(a: int, b: int) -> int:
    """iAlignUp (cuda_utils.h:160-163)."""
    return a - a % b + b if a % b else a


# ------------------------------------------------------------------ runtime

def device_count() -> int:
    n = C.c_int()
    check(_lib.surfhip_get_device_count(C.byref(n)), "device_count")
    return n.value


def set_device(dev: int) -> None:
    check(_lib.surfhip_set_device(dev), "set_device")


def device_name(dev: int = 0):
    buf = C.create_string_buffer(256)
    cu = C.c_int()
    check(_lib.surfhip_device_name(dev, buf, 256, C.byref(cu)), "device_name")
    return buf.value.decode(), cu.value


def synchronize() -> None:
    check(_lib.surfhip_device_synchronize(), "synchronize")


class DeviceBuffer:
    """An HBM allocation owned by Python (surfhip_malloc / surfhip_free)."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        check(_lib.surfhip_malloc(C.byref(p), max(self.nbytes, 1)), f"malloc({nbytes})")
        self.ptr = p.value

    def upload(self, arr: np.ndarray, offset: int = 0) -> None:
        a = np.ascontiguousarray(arr)
        assert offset + a.nbytes <= self.nbytes
        check(_lib.surfhip_memcpy(self.ptr + offset, a.ctypes.data, a.nbytes, H2D), "upload")

    def download(self, dtype, count: int, offset: int = 0) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        assert offset + out.nbytes <= self.nbytes
        if out.nbytes:
            check(_lib.surfhip_memcpy(out.ctypes.data, self.ptr + offset, out.nbytes, D2H), "download")
        return out

    def zero(self) -> None:
        check(_lib.surfhip_memset(self.ptr, 0, self.nbytes), "memset")

    def free(self) -> None:
        if self.ptr:
            _lib.surfhip_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def download_ptr(ptr: int, dtype, count: int) -> np.ndarray:
    out = np.empty(count, dtype=dtype)
    if out.nbytes:
        check(_lib.surfhip_memcpy(out.ctypes.data, ptr, out.nbytes, D2H), "download")
    return out


def event_create() -> int:
    e = C.c_void_p()
    check(_lib.surfhip_event_create(C.byref(e)), "event_create")
    return e.value


def event_destroy(event: int) -> None:
    check(_lib.surfhip_event_destroy(event), "event_destroy")


def stream_wait_event(stream, event: int) -> None:
    """Make `stream` (a hipStream_t handle) wait for the event's last record."""
    check(_lib.surfhip_stream_wait_event(stream, event), "stream_wait_event")


STREAM_MODES = {"copy": 0, "read": 1, "write": 2}


def stream_run(mode: str, src: int | None, dst: int | None, nbytes: int, stream=None) -> int:
    """One launch of the HBM stream-rate kernel (surfhip_stream_run); returns
    the HBM bytes it moves (copy: read + write)."""
    m = STREAM_MODES[mode]
    check(_lib.surfhip_stream_run(m, src, dst, nbytes, stream), f"stream_run({mode})")
    return int(_lib.surfhip_stream_bytes(m, nbytes))


def upload_ptr(ptr: int, arr: np.ndarray) -> None:
    a = np.ascontiguousarray(arr)
    if a.nbytes:
        check(_lib.surfhip_memcpy(ptr, a.ctypes.data, a.nbytes, H2D), "upload")


# ---------------------------------------------------------------- detector

def make_param(noctaves=4, thresh=0.2, doubled=False, init_mask_size=9, sampling_step=2,
               upright=False, extend=False, desc_wsz=4) -> SurfParam:
    """Surfor::init parameter derivation (surf.cpp:60-79); defaults of surf.h:27-29."""
    p = SurfParam()
    check(_lib.surfhip_make_param(C.byref(p), noctaves, C.c_float(thresh), int(doubled), init_mask_size,
                                  sampling_step, int(upright), int(extend), desc_wsz), "make_param")
    return p


class Detector:
    """One geometry + SurfParam + batch scratch on the current device."""

    def __init__(self, param: SurfParam, width: int, height: int, max_batch: int = 1,
                 max_pts: int = 16384, cand_cap: int = 0, stream: int | None = None):
        self.param = param
        self.width, self.height = width, height
        self.max_batch, self.max_pts = max_batch, max_pts
        h = C.c_void_p()
        check(_lib.surfhip_detector_create(C.byref(h), C.byref(param), width, height, max_batch, max_pts,
                                           cand_cap, stream), "detector_create")
        self.h = h.value

    @property
    def nfeatures(self) -> int:
        return self.param.nfeatures

    def set_stream(self, stream) -> None:
        check(_lib.surfhip_detector_set_stream(self.h, stream), "set_stream")

    def set_profiling(self, on: bool) -> None:
        check(_lib.surfhip_detector_set_profiling(self.h, int(on)), "set_profiling")

    def time_hessian(self, on: bool) -> None:
        """Record the Hessian launches of the following batches with HIP events
        in their in-step (pipelined) arrangement."""
        check(_lib.surfhip_detector_time_hessian(self.h, int(on)), "time_hessian")

    def hessian_times(self) -> list:
        """Milliseconds of each recorded batch's whole Hessian stage, from its
        fork to the end of its last kernel on either stream (and reset)."""
        ms = (C.c_float * 64)()
        n = _i(0)
        check(_lib.surfhip_detector_hessian_times(self.h, ms, 64, C.byref(n)), "hessian_times")
        return [float(ms[k]) for k in range(n.value)]

    def stage_times(self) -> dict:
        ms = (C.c_float * NSTAGE)()
        check(_lib.surfhip_detector_stage_times(self.h, ms), "stage_times")
        return dict(zip(STAGES, [float(v) for v in ms]))

    def detect_batch(self, frames_ptr: int, nframes: int, pitch: int, stride: int,
                     points_ptr: int, desc_ptr: int | None, counts_ptr: int) -> None:
        check(_lib.surfhip_detect_batch(self.h, frames_ptr, nframes, pitch, stride, points_ptr,
                                        desc_ptr, counts_ptr), "detect_batch")

    def detect_batch_next(self, frames_ptr: int, nframes: int, pitch: int, stride: int, points_ptr: int,
                          desc_ptr: int | None, counts_ptr: int, next_ptr: int | None, next_nframes: int = 0,
                          next_pitch: int = 0, next_stride: int = 0) -> None:
        """detect_batch, with the next batch's integral computed beside this
        batch's describe stage (surfhip_detect_batch_next)."""
        check(_lib.surfhip_detect_batch_next(self.h, frames_ptr, nframes, pitch, stride, points_ptr, desc_ptr,
                                             counts_ptr, next_ptr, next_nframes, next_pitch, next_stride),
              "detect_batch_next")

    def set_describe_event(self, event: int | None) -> None:
        """Record `event` (event_create) before each describe stage
        (surfhip_detector_set_describe_event); None stops it."""
        check(_lib.surfhip_detector_set_describe_event(self.h, event), "set_describe_event")

    def drain(self) -> None:
        """Order the side stream's pending prefetch before the detector
        stream's later work (surfhip_detector_drain)."""
        check(_lib.surfhip_detector_drain(self.h), "drain")

    def run_integral(self, frames_ptr, nframes, pitch, stride) -> None:
        check(_lib.surfhip_run_integral(self.h, frames_ptr, nframes, pitch, stride), "run_integral")

    def run_hessian(self, nframes) -> None:
        check(_lib.surfhip_run_hessian(self.h, nframes), "run_hessian")

    def candidates(self, nframes: int) -> np.ndarray:
        out = np.zeros(nframes, np.int32)
        rc = _lib.surfhip_detector_candidates(self.h, out.ctypes.data_as(C.POINTER(C.c_int)), nframes)
        if rc not in (0, -3):
            check(rc, "candidates")
        return out

    def truncated(self) -> bool:
        """Whether the last batch dropped candidates at the candidate capacity."""
        t = C.c_int()
        check(_lib.surfhip_detector_status(self.h, C.byref(t)), "status")
        return bool(t.value)

    def capacity(self) -> int:
        c = C.c_int()
        check(_lib.surfhip_detector_capacity(self.h, C.byref(c)), "capacity")
        return c.value

    def workspace(self):
        ii, iis, rs, rss = C.c_void_p(), C.c_size_t(), C.c_void_p(), C.c_size_t()
        check(_lib.surfhip_detector_workspace(self.h, C.byref(ii), C.byref(iis), C.byref(rs), C.byref(rss)),
              "workspace")
        return ii.value, iis.value, rs.value, rss.value

    def geometry(self):
        iwhp = (C.c_int * 3)()
        swhp = (C.c_int * 24)()
        ooff = (C.c_longlong * 8)()
        osize = (C.c_int * 8)()
        check(_lib.surfhip_detector_geometry(self.h, iwhp, swhp, ooff, osize), "geometry")
        return (tuple(iwhp), [tuple(swhp[3 * o:3 * o + 3]) for o in range(8)], list(ooff), list(osize))

    def hessian_bytes_per_frame(self) -> int:
        return int(_lib.surfhip_hessian_bytes_per_frame(self.h))

    def hessian_kernels(self) -> str:
        """The Hessian stage's kernels of this detector's plan (surfhip_hessian_plan)."""
        buf = C.create_string_buffer(256)
        n = _lib.surfhip_hessian_plan(self.h, buf, len(buf))
        if n < 0:
            check(n, "hessian_plan")
        if n >= len(buf):                     # the plan text was cut: ask again with room for all of it
            buf = C.create_string_buffer(n + 1)
            check(min(0, _lib.surfhip_hessian_plan(self.h, buf, len(buf))), "hessian_plan")
        return buf.value.decode()

    def slab_bytes(self, nframes: int, total: int, desc: bool = True) -> int:
        return int(_lib.surfhip_slab_bytes(nframes, total, self.nfeatures if desc else 0))

    def batch_total(self, nframes: int) -> int:
        t = C.c_int()
        check(_lib.surfhip_batch_total(self.h, nframes, C.byref(t)), "batch_total")
        return t.value

    def pack_slab(self, points_ptr, desc_ptr, counts_ptr, nframes, slab_ptr) -> None:
        check(_lib.surfhip_pack_slab(self.h, points_ptr, desc_ptr, counts_ptr, nframes, slab_ptr), "pack_slab")

    def pack_slab_cap(self, points_ptr, desc_ptr, counts_ptr, nframes, slab_ptr, cap_bytes) -> None:
        """Pack into a buffer of a capacity agreed once (no host sync); a batch
        that does not fit sets SLAB_OVERFLOW in the slab's flags."""
        check(_lib.surfhip_pack_slab_cap(self.h, points_ptr, desc_ptr, counts_ptr, nframes, slab_ptr, cap_bytes),
              "pack_slab_cap")

    def detect(self, image_ptr: int, pitch: int, points_ptr: int, max_pts: int, desc: bool = True):
        """Surfor::detectAndCompute semantics for one frame (synchronous)."""
        n = C.c_int()
        dptr = C.c_void_p()
        check(_lib.surfhip_detect(self.h, image_ptr, pitch, points_ptr, max_pts, C.byref(n), C.byref(dptr),
                                  int(desc)), "detect")
        return n.value, dptr.value

    def close(self) -> None:
        if self.h:
            _lib.surfhip_detector_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------- reference-shaped host API

class SurfData:
    """surf_structures.h:34-40 + initSurfData/freeSurfData (surf.cpp:10-36)."""

    def __init__(self, max_pts: int, host: bool = True, dev: bool = True):
        self.num_pts = 0
        self.max_pts = max_pts
        self.h_data = np.zeros(max_pts, POINT_DTYPE) if host else None
        self.d_data = DeviceBuffer(48 * max_pts) if dev else None

    def free(self) -> None:
        if self.d_data is not None:
            self.d_data.free()
        self.h_data = None
        self.num_pts = 0
        self.max_pts = 0


def initSurfData(max_pts: int, host: bool, dev: bool) -> SurfData:  # noqa: N802 (reference name)
    return SurfData(max_pts, host, dev)


def freeSurfData(data: SurfData) -> None:  # noqa: N802
    data.free()


class Surfor:
    """Mirror of surf::Surfor (surf.h:17-62) over the C-ABI."""

    def __init__(self):
        self.its = None
        self.whp = (0, 0, 0)
        self._det = None

    def init(self, noctaves, thresh=0.2, doubled=False, init_mask_size=9, sampling_step=2,
             upright=False, extend=False, desc_wsz=4, width=-1, height=-1):
        self.its = make_param(noctaves, thresh, doubled, init_mask_size, sampling_step, upright, extend,
                              desc_wsz)
        self.whp = (width, height, align_up(width, 128) if width > 0 else -1)
        self._det = None
        self._max_pts = 0

    def _detector(self, w, h, max_pts):
        if self._det is None or (self._det.width, self._det.height) != (w, h) or self._max_pts < max_pts:
            if self._det is not None:
                self._det.close()
            self._det = Detector(self.its, w, h, 1, max_pts)
            self._max_pts = max_pts
        return self._det

    def detectAndCompute(self, image_ptr: int, result: SurfData, whp0, desc: bool = True):  # noqa: N802
        """surf.cpp:205-355.  Returns the new descriptor device pointer (or None)."""
        w, h, p = whp0
        det = self._detector(w, h, result.max_pts)
        n, dptr = det.detect(image_ptr, p, result.d_data.ptr, result.max_pts, desc)
        result.num_pts = n
        if result.h_data is not None and n > 0:
            # surf.cpp:335-342: the first 6 (7 if rotated descriptors) fields
            nf = 7 if (desc and not self.its.upright) else 6
            tmp = download_ptr(result.d_data.ptr, POINT_DTYPE, n)
            for name in POINT_DTYPE.names[:nf]:
                result.h_data[name][:n] = tmp[name]
        return dptr if desc else None


    def match(self, data1: SurfData, data2: SurfData, features1: int, features2: int) -> None:
        """Surfor::match (surf.cpp:418-428): findMaxCorr of data1 against
        data2 on the device, then the five match fields (score, match,
        match_x, match_y, ambiguity) copied to data1.h_data."""
        match_points(data1.d_data.ptr, data2.d_data.ptr, features1, features2, data1.num_pts,
                     data2.num_pts, self.its.nfeatures)
        synchronize()
        if data1.h_data is not None and data1.num_pts > 0:
            tmp = download_ptr(data1.d_data.ptr, POINT_DTYPE, data1.num_pts)
            for name in ("score", "match", "match_x", "match_y", "ambiguity"):
                data1.h_data[name][:data1.num_pts] = tmp[name]


MATCH_FULL_TAIL = 1


def match_points(pts1_ptr: int, pts2_ptr: int, feat1_ptr: int, feat2_ptr: int, n1: int, n2: int,
                 nfeatures: int, flags: int = 0, scratch_ptr: int | None = None, stream=None) -> None:
    """surfhip_match (cuFindMaxCorr, surfd.cu:3554-3566), asynchronous on
    `stream` (a raw hipStream_t or None for the null stream)."""
    check(_lib.surfhip_match(pts1_ptr, pts2_ptr, feat1_ptr, feat2_ptr, n1, n2, nfeatures, flags,
                             scratch_ptr, stream), "surfhip_match")


def match_scratch_bytes(n1: int, n2: int, flags: int = 0) -> int:
    return int(_lib.surfhip_match_scratch(n1, n2, flags))


# ---------------------------------------------------------------- frames

def synth_frames(n: int, width: int, height: int, pitch: int | None = None, first: int = 0,
                 nblobs: int = 0, nthreads: int = 0) -> np.ndarray:
    """Deterministic synthetic frames (seed 0x5EED0000 + index), [n, H, pitch] u8."""
    pitch = pitch or align_up(width, 128)
    out = np.zeros((n, height, pitch), np.uint8)
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    rc = _syn.surf_synth_frames(out.ctypes.data, n, width, height, pitch, height * pitch, first, nblobs, nthreads)
    if rc:
        raise SurfError(f"synth_frames failed ({rc})")
    return out


def read_pgm(path: str, pitch: int | None = None) -> np.ndarray:
    w, h = C.c_int(), C.c_int()
    if _syn.surf_pgm_info(path.encode(), C.byref(w), C.byref(h)) < 0:
        raise SurfError(f"not a P5/255 PGM: {path}")
    pitch = pitch or align_up(w.value, 128)
    out = np.zeros((h.value, pitch), np.uint8)
    if _syn.surf_pgm_read(path.encode(), out.ctypes.data, pitch):
        raise SurfError(f"short PGM: {path}")
    return out, w.value, h.value


def downsample2(img: np.ndarray, w: int, h: int) -> np.ndarray:
    src = np.ascontiguousarray(img)
    pitch = align_up(w // 2, 128)
    out = np.zeros((h // 2, pitch), np.uint8)
    _syn.surf_downsample2(src.ctypes.data, w, h, src.shape[1], out.ctypes.data, pitch)
    return out


SLAB_TRUNCATED, SLAB_OVERFLOW = 1, 2      # slab header flags (include/surfhip.h)


def slab_flags(buf: np.ndarray) -> int:
    return int(np.ascontiguousarray(buf[:16]).view(np.uint8).view(np.int32)[3])


def parse_slab(buf: np.ndarray):
    """Host view of one compacted result slab (see include/surfhip.h):
    returns (counts[nframes], points[total], desc[total, nf] or None)."""
    b = np.ascontiguousarray(buf).view(np.uint8)
    nframes, total, nf, _ = (int(v) for v in b[:16].view(np.int32))
    counts = b[16:16 + 4 * nframes].view(np.int32).copy()
    head = 16 + ((4 * nframes + 15) & ~15)
    pts = b[head:head + 48 * total].view(POINT_DTYPE).copy()
    desc = None
    if nf:
        o = head + 48 * total
        desc = b[o:o + 4 * total * nf].view(np.float32).reshape(total, nf).copy()
    return counts, pts, desc


def build_slab(counts: np.ndarray, pts: np.ndarray, desc) -> np.ndarray:
    """Host-side builder of the same format (used by the CPU tests)."""
    nframes, total = len(counts), int(counts.sum())
    nf = 0 if desc is None else desc.shape[1]
    head = 16 + ((4 * nframes + 15) & ~15)
    out = np.zeros(head + total * (48 + 4 * nf), np.uint8)
    out[:16].view(np.int32)[:] = (nframes, total, nf, 0)
    out[16:16 + 4 * nframes].view(np.int32)[:] = counts
    out[head:head + 48 * total] = np.ascontiguousarray(pts[:total]).view(np.uint8)
    if nf:
        out[head + 48 * total:] = np.ascontiguousarray(desc[:total], dtype=np.float32).view(np.uint8).ravel()
    return out


# ------------------------------------------------------ multi-GPU exchange

COMM_PATH = os.path.join(_HERE, "libsurfcomm.so")
COMM_ID_BYTES = 128
_comm_lib = None


def _comm():
    """libsurfcomm.so (include/surfhip_comm.h), loaded on first use so that
    single-GPU callers never load RCCL."""
    global _comm_lib
    if _comm_lib is None:
        if not os.path.exists(COMM_PATH):
            raise ImportError(f"surf_amd: {COMM_PATH} is missing -- run `make -C cuda-surf_amd`")
        L = C.CDLL(COMM_PATH)
        for name, res, args in (("surfhip_comm_unique_id", _i, [_vp]),
                                ("surfhip_comm_init", _i, [C.POINTER(_vp), _i, _i, _vp]),
                                ("surfhip_comm_destroy", _i, [_vp]),
                                ("surfhip_comm_rank", _i, [_vp, C.POINTER(_i), C.POINTER(_i)]),
                                ("surfhip_allgather", _i, [_vp, _vp, _sz, _vp, _vp]),
                                ("surfhip_allreduce_sum_i64", _i, [_vp, _vp, _i, _vp]),
                                ("surfhip_comm_last_error", _i, [])):
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _comm_lib = L
    return _comm_lib


def comm_unique_id() -> bytes:
    buf = C.create_string_buffer(COMM_ID_BYTES)
    rc = _comm().surfhip_comm_unique_id(buf)
    check(rc, f"comm_unique_id (rccl {_comm().surfhip_comm_last_error()})")
    return buf.raw


class Comm:
    """One RCCL communicator of this process's GPU (surfhip_comm_*).  The
    128-byte id comes from comm_unique_id() on one rank, shared out of band
    (the bench broadcasts it over its torch.distributed group)."""

    def __init__(self, nranks: int, rank: int, uid: bytes):
        assert len(uid) == COMM_ID_BYTES
        h = C.c_void_p()
        idb = C.create_string_buffer(uid, COMM_ID_BYTES)
        rc = _comm().surfhip_comm_init(C.byref(h), nranks, rank, idb)
        check(rc, f"comm_init (rccl {_comm().surfhip_comm_last_error()})")
        self.h, self.nranks, self.rank = h.value, nranks, rank

    def allgather(self, send_ptr: int, nbytes: int, recv_ptr: int, stream=None) -> None:
        rc = _comm().surfhip_allgather(self.h, send_ptr, nbytes, recv_ptr, stream)
        check(rc, f"allgather (rccl {_comm().surfhip_comm_last_error()})")

    def allreduce_sum_i64(self, ptr: int, n: int, stream=None) -> None:
        rc = _comm().surfhip_allreduce_sum_i64(self.h, ptr, n, stream)
        check(rc, f"allreduce (rccl {_comm().surfhip_comm_last_error()})")

    def close(self) -> None:
        if self.h:
            _comm().surfhip_comm_destroy(self.h)
            self.h = None


class Ingest:
    """Pipelined host-frame ring over one Detector (surfhip_ingest_*):
    `acquire()` gives a pinned u8 view [max_batch, H, pitch] to fill,
    `submit(n)` queues H2D + detect + pack, `collect()` returns the oldest
    batch's result slab (a host copy; parse with parse_slab)."""

    def __init__(self, det: "Detector", depth: int = 2):
        self.det, self.depth = det, depth
        h = C.c_void_p()
        check(_lib.surfhip_ingest_create(C.byref(h), det.h, depth), "ingest_create")
        self.handle = h.value

    def acquire(self) -> np.ndarray:
        p, pitch, stride = C.c_void_p(), C.c_int(), C.c_size_t()
        check(_lib.surfhip_ingest_acquire(self.handle, C.byref(p), C.byref(pitch), C.byref(stride)),
              "ingest_acquire")
        n = self.det.max_batch * stride.value
        buf = (C.c_uint8 * n).from_address(p.value)
        return np.frombuffer(buf, np.uint8).reshape(self.det.max_batch, self.det.height, pitch.value)

    def submit(self, nframes: int) -> None:
        check(_lib.surfhip_ingest_submit(self.handle, nframes), "ingest_submit")

    def collect(self, copy: bool = True) -> np.ndarray:
        """copy=False returns a view of the pinned slab, valid until this
        slot is collected again (`depth` collects later)."""
        p, n = C.c_void_p(), C.c_size_t()
        check(_lib.surfhip_ingest_collect(self.handle, C.byref(p), C.byref(n)), "ingest_collect")
        v = np.frombuffer((C.c_uint8 * n.value).from_address(p.value), np.uint8)
        return v.copy() if copy else v

    def pending(self) -> int:
        n = C.c_int()
        check(_lib.surfhip_ingest_pending(self.handle, C.byref(n)), "ingest_pending")
        return n.value

    def close(self) -> None:
        if self.handle:
            check(_lib.surfhip_ingest_destroy(self.handle), "ingest_destroy")
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


DUMP_MAGIC = b"SURFKPD1"
DUMP_HEADER_DTYPE = np.dtype([("magic", "S8"), ("header_bytes", "<u4"), ("version", "<u4"),
                              ("width", "<u4"), ("height", "<u4"), ("nframes", "<u4"),
                              ("nfeatures", "<u4"), ("total", "<u8"), ("slab_bytes", "<u8"),
                              ("first_frame", "<u8"), ("thresh", "<f4"), ("noctaves", "u1"),
                              ("upright", "u1"), ("extend", "u1"), ("doubled", "u1")])
assert DUMP_HEADER_DTYPE.itemsize == 64


def dump_append(path: str, slab: np.ndarray, width: int, height: int, param: SurfParam,
                first_frame: int = 0) -> None:
    """Append one result slab as a record of the keypoint file (surfhip_dump_append)."""
    b = np.ascontiguousarray(slab, dtype=np.uint8)
    check(_lib.surfhip_dump_append(path.encode(), b.ctypes.data, b.nbytes, width, height,
                                   C.byref(param), first_frame), "dump_append")


def read_dump(path: str):
    """Records of a keypoint file: list of (header dict, counts, points, desc or None)."""
    raw = np.fromfile(path, np.uint8)
    out, o = [], 0
    while o < raw.size:
        if raw.size - o < 64:
            raise ValueError(f"{path}: truncated record header at byte {o}")
        h = raw[o:o + 64].view(DUMP_HEADER_DTYPE)[0]
        if h["magic"] != DUMP_MAGIC or h["header_bytes"] != 64 or h["version"] != 1:
            raise ValueError(f"{path}: bad record header at byte {o}")
        n = int(h["slab_bytes"])
        if raw.size - o - 64 < n:
            raise ValueError(f"{path}: truncated slab at byte {o + 64}")
        counts, pts, desc = parse_slab(raw[o + 64:o + 64 + n])
        if len(counts) != h["nframes"] or len(pts) != h["total"]:
            raise ValueError(f"{path}: record at byte {o} disagrees with its slab")
        out.append(({k: (h[k].item() if k != "magic" else bytes(h[k])) for k in DUMP_HEADER_DTYPE.names},
                    counts, pts, desc))
        o += 64 + n
    return out


from . import dist  # noqa: E402  (multi-GPU sharding + slab all-gather helpers)
