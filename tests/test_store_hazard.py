"""The gfx950 store-data hazard: a 12- or
16-B store's data VGPRs must not be rewritten by a VALU instruction within 1
wait state (buffer store, SGPR soffset) or 2 (constant soffset, global
store) -- measured by tools/ubench/store_hazard.hip; LLVM's hazard recognizer
gives 0 and 1.  CPU tests: the scanner's rule on a hand-written listing, and
no store of the built libsurfhip.so breaking it."""
from __future__ import annotations

import importlib.util
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "cuda-surf_amd", "libsurfhip.so")


def _scanner():
    spec = importlib.util.spec_from_file_location("store_hazard_scan",
                                                  os.path.join(REPO, "tools", "store_hazard_scan.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


LISTING = """\
_Zk_sgpr_next:
\tbuffer_store_dwordx4 v[2:5], v10, s[16:19], s70 offen nt
\tv_add_u32_e32 v3, s71, v30
_Zk_sgpr_one:
\tbuffer_store_dwordx4 v[2:5], v10, s[16:19], s70 offen nt
\tv_mov_b32_e32 v40, v1
\tv_add_u32_e32 v3, s71, v30
_Zk_const_one:
\tbuffer_store_dwordx4 v[2:5], v10, s[16:19], 0 offen nt
\ts_nop 0
\tv_mov_b32_e32 v5, 0
_Zk_const_two:
\tbuffer_store_dwordx4 v[2:5], v10, s[16:19], 0 offen nt
\tv_mov_b32_e32 v40, v1
\tv_mov_b32_e32 v41, v1
\tv_mov_b32_e32 v5, 0
_Zk_global_one:
\tglobal_store_dwordx4 v[8:9], v[40:43], off
\tv_mov_b32_e32 v44, v1
\tv_mov_b32_e32 v41, -1
_Zk_x2_next:
\tbuffer_store_dwordx2 v[2:3], v10, s[16:19], 0 offen
\tv_mov_b32_e32 v2, 0
_Zk_branch:
\tbuffer_store_dwordx4 v[2:5], v10, s[16:19], 0 offen
\ts_branch .LBB0_1
\tv_mov_b32_e32 v2, 0
.LBB0_1:
\tv_mov_b32_e32 v3, 0
_Zk_branch_far:
\tbuffer_store_dwordx4 v[2:5], v10, s[16:19], 0 offen
\ts_branch .LBB0_2
.LBB0_2:
\ts_nop 0
\tv_mov_b32_e32 v3, 0
"""


def test_scanner_rule(tmp_path):
    sc = _scanner()
    p = tmp_path / "k.s"
    p.write_text(LISTING)
    counts, hits = sc.scan(str(p), None)
    flagged = {k for k, v in counts.items() if v[1]}
    # (_Zk_branch: the overwrite one wait state away through the s_branch;
    # _Zk_branch_far: two)
    assert flagged == {"_Zk_sgpr_next", "_Zk_const_one", "_Zk_global_one", "_Zk_branch"}, flagged
    assert sc.need("s70") == 1 and sc.need("vcc_lo") == 1 and sc.need("0") == 2 and sc.need("-") == 2


@pytest.mark.skipif(not os.path.exists(LIB), reason="libsurfhip.so not built")
def test_built_library_has_no_exposed_wide_store(tmp_path):
    sc = _scanner()
    files = sc.disassemble_lib(LIB, str(tmp_path))
    assert files, "no gfx950 code object found in libsurfhip.so"
    total, nstores, where = 0, 0, []
    for f in files:
        counts, hits = sc.scan(f, None)
        for k, (ns, nh) in counts.items():
            nstores += ns
            total += nh
            if nh:
                where.append((k[:80], hits[k][:3]))
    assert nstores > 100, nstores           # the scanner saw the kernels' wide stores
    assert total == 0, where
