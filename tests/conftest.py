"""Shared test setup.

- registers the ``gpu`` marker (tests that need an MI355X);
- loads the product package ``cuda-surf_amd`` (as ``surf_amd``) and the CPU
  oracle binding ``oracle/oracle.py`` (test infrastructure);
- never imports torch at module level: a GPU test process must hold a single
  HIP runtime (ours, /opt/rocm), see cuda-surf_amd/__init__.py.
"""
from __future__ import annotations

import importlib.util
import os
import subprocess
import sys

import numpy as np
import pytest


# The parity tests run small batches; keep them on the streaming Hessian
# kernels the batched path uses (a detector with max_batch <= 8 would pick the
# gather kernel); tests of the gather plan set SURFHIP_HESS_GATHER=1 themselves.
os.environ.setdefault("SURFHIP_HESS_GATHER", "0")
# ... and on k_describe_u2 (the batched default; batches <= 8 frames pick
# k_describe_ur): tests of the small-batch default unset it themselves.
os.environ.setdefault("SURFHIP_DESC_UR", "0")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
REF_DATA = "/root/reference/data"       # present in the build container only


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (gfx950) GPU")


def _ensure_built():
    libs = [os.path.join(REPO, "cuda-surf_amd", n) for n in ("libsurfhip.so", "libsurfsynth.so")]
    if not all(os.path.exists(p) for p in libs):
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "cuda-surf_amd")])


def load_surf_amd():
    if "surf_amd" in sys.modules:
        return sys.modules["surf_amd"]
    _ensure_built()
    pkg = os.path.join(REPO, "cuda-surf_amd")
    spec = importlib.util.spec_from_file_location("surf_amd", os.path.join(pkg, "__init__.py"),
                                                  submodule_search_locations=[pkg])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["surf_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_oracle():
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # noqa: E402
    return oracle


@pytest.fixture(scope="session")
def surf():
    return load_surf_amd()


@pytest.fixture(scope="session")
def orc():
    return load_oracle()


def gpu_available() -> bool:
    try:
        s = load_surf_amd()
        return s.device_count() > 0
    except Exception:
        return False


# ------------------------------------------------------------ comparisons

KEY_FIELDS = ("o", "y", "x", "scale")


def canonical(pts: np.ndarray) -> np.ndarray:
    """Sort keypoints by (octave, y, x, scale) -- SURVEY.md A8."""
    idx = np.lexsort(tuple(pts[k] for k in reversed(KEY_FIELDS)))
    return idx


def assert_points_equal(a: np.ndarray, b: np.ndarray, fields=("x", "y", "scale", "o", "strength", "laplace")):
    assert len(a) == len(b), f"keypoint count {len(a)} != {len(b)}"
    for f in fields:
        va, vb = a[f], b[f]
        if va.dtype.kind == "f":
            same = (va.view(np.uint32) == vb.view(np.uint32))
        else:
            same = va == vb
        if not same.all():
            i = int(np.argmin(same))
            raise AssertionError(f"field {f} differs at {i}: {va[i]!r} vs {vb[i]!r} "
                                 f"({(~same).sum()} of {len(a)} differ)")


def desc_l2(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    return np.sqrt(((a.astype(np.float64) - b.astype(np.float64)) ** 2).sum(axis=1))
