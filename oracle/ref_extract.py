#!/usr/bin/env python3
"""Build oracle/_ref/libref_host.so from the reference's own host C++.

TEST INFRASTRUCTURE ONLY (pins the oracle; never loaded by the product).
surfd.cu cannot be compiled here (nvcc / CUDA headers absent), but
three pieces of it are plain host C++ that g++ compiles as they stand:

  * surfd.cu:3082-3130  hSolveLinearSystem  (the host twin of the device
                        solveLinearSystem, surfd.cu:835-887)
  * surfd.cu:3133-3186  hFitQuadrat's body  (the host twin of fitQuadrat,
                        surfd.cu:942-988)
  * surfd.cu:2833-2866  the per-scale Hessian parameter recurrence of
                        cuCalcHessianMulti (masks, borders, norms, x2/x3/x4)
  * surfd.h:9-10        MAX_SCALE / MAX_OCTAVE
  * surf.cpp:358-371    initLut's two table loops (the setLut uploads left out)
  * surf.cpp:240, 261, 269  the octave loop's statements that start the mask
                        recurrence and compute border1 (octave 0 / octaves > 0);
                        the harness runs them in surf.cpp:241-293's loop order
                        around cuCalcHessianMulti's parameter block
  * surf.cpp:67-79      Surfor::init's SurfParam derivation (and whp)
  * surf.cpp:377-392    allocMemory's geometry (iwhp, swhps, osizes, tot_osize)
  * cuda_utils.h:160-163  iAlignUp, which both of the above call
  * surfd.cu:3060-3076  cuFindMaximumWithInterp's NMS borders (mborders) and
                        grid extent; the dim3 grid's three argument expressions
                        are taken as text and evaluated into ints (no dim3 is
                        stood in for)

The text is copied verbatim from /root/reference at build time into
oracle/_ref/ (git-ignored) and wrapped in extern "C" harness functions whose
parameter lists are ours.  One CUDA type IS stood in for: hFitQuadrat's body
reads swhps[o].z, and its parameter is declared with our `struct ref_dims
{int x, y, z;}` where the reference has CUDA's `int3` (surfd.cu's signature,
not its body, names int3); the fit pin therefore rests on that stand-in
(VERDICT r05), while hSolveLinearSystem and the parameter blocks compile
with no stand-in.  No reference header or library is stood in for.  Compiled with
g++ -ffp-contract=off: one rounding per written float op, the semantics the
oracle restates.  tests/test_oracle.py compares the oracle's solve3,
fit_quadratic and or_octave_params with these bit for bit.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("SURF_REFERENCE", "/root/reference")
OUT = os.path.join(HERE, "_ref")


def _block(lines, start):
    """Lines from `start` through the brace that closes the first '{'."""
    depth, seen = 0, False
    for i in range(start, len(lines)):
        depth += lines[i].count("{") - lines[i].count("}")
        seen = seen or "{" in lines[i]
        if seen and depth == 0:
            return lines[start:i + 1], i
    raise ValueError("unbalanced block")


def _find(lines, needle, lo=0):
    for i in range(lo, len(lines)):
        if needle in lines[i]:
            return i
    raise ValueError(f"not found: {needle!r}")


def extract():
    cu = open(os.path.join(REF, "surfd.cu")).read().split("\n")
    hh = open(os.path.join(REF, "surfd.h")).read().split("\n")
    defs = [l for l in hh[:20] if l.startswith("#define MAX_SCALE") or l.startswith("#define MAX_OCTAVE")]
    assert len(defs) == 2, defs
    s = _find(cu, "void hSolveLinearSystem(float* solution, float sq[3][3], int size)")
    solve, _ = _block(cu, s)
    f = _find(cu, "float hFitQuadrat(")
    fit, _ = _block(cu, f)
    fit_body = fit[1:]                                   # from the opening brace
    p0 = _find(cu, "void cuCalcHessianMulti(")
    a = _find(cu, "const int nscale = max_scale - init_scale;", p0)
    b = _find(cu, "init_mask_size = mask_sizes[nscale - 1];", a)
    params = cu[a:b + 1]
    return defs, solve, fit_body, params, (s + 1, f + 1, a + 1, b + 1)


def extract_host():
    """surf.cpp: initLut's loops and the border statements of detectAndCompute."""
    cpp = open(os.path.join(REF, "surf.cpp")).read().split("\n")
    li = _find(cpp, "void Surfor::initLut()")
    l1 = _find(cpp, "for (int n = 0; n < 83; n++)", li)
    loop1, e1 = _block(cpp, l1)
    l2 = _find(cpp, "for (int n = 0; n < 40; n++)", e1)
    loop2, _ = _block(cpp, l2)
    d0 = _find(cpp, "void Surfor::detectAndCompute(")
    m = _find(cpp, "int mask_size = its.init_lobe - 2;", d0)
    bo = _find(cpp, "border1 = ((3 * (mask_size + 4 * octave)) / 2) / (its.sampling * octave) + 1;", m)
    b0 = _find(cpp, "border1 = ((3 * (mask_size + 6 * octave)) / 2) / (its.sampling * octave) + 1;", m)
    return {"loop1": loop1, "loop2": loop2, "mask": cpp[m], "border_o": cpp[bo], "border_0": cpp[b0],
            "where": (l1 + 1, l2 + 1, m + 1, bo + 1, b0 + 1)}


def extract_more():
    """surf.cpp Surfor::init / allocMemory, cuda_utils.h iAlignUp, surfd.cu's
    NMS border loop and grid extent."""
    cpp = open(os.path.join(REF, "surf.cpp")).read().split("\n")
    cu = open(os.path.join(REF, "surfd.cu")).read().split("\n")
    cuh = open(os.path.join(REF, "cuda_utils.h")).read().split("\n")
    a = _find(cuh, "inline int iAlignUp(const int a, const int b)")
    align, _ = _block(cuh, a)
    si = _find(cpp, "void Surfor::init(")
    i0 = _find(cpp, "whp.x = _width;", si)
    i1 = _find(cpp, "its.nfeatures = _desc_wsz * _desc_wsz * its.orient_size;", i0)
    init = cpp[i0:i1 + 1]
    am = _find(cpp, "int Surfor::allocMemory(")
    g0 = _find(cpp, "iwhp.x = its.doubled ? w + w - 1 : w + 1;", am)
    lp = _find(cpp, "for (int i = 0, j = 1; j < its.noctaves; i++, j++)", g0)
    loop, g1 = _block(cpp, lp)
    geo = cpp[g0:g1 + 1]
    fm = _find(cu, "void cuFindMaximumWithInterp(")
    dx = _find(cu, "#define DX 16", fm)
    dy = _find(cu, "#define DY 16", fm)
    n0 = _find(cu, "int n = 0, b = 0, maxw = 0, maxh = 0;", fm)
    nl = _find(cu, "for (int k = 1; k < its.max_scale - 1; k += 2)", n0)
    nloop, _ = _block(cu, nl)
    gr = _find(cu, "dim3 grid(", nl)
    gline = cu[gr].strip()
    assert gline.startswith("dim3 grid(") and gline.endswith(");"), gline
    args, depth, cur = [], 0, ""
    for ch in gline[len("dim3 grid("):-2]:
        if ch == "," and depth == 0:
            args.append(cur.strip()); cur = ""; continue
        depth += ch == "("
        depth -= ch == ")"
        cur += ch
    args.append(cur.strip())
    assert len(args) == 3, args
    return {"align": align, "init": init, "geo": geo,
            "nms": [cu[dx], cu[dy], cu[n0], cu[n0 + 1]] + nloop, "grid": args,
            "where": (a + 1, i0 + 1, i1 + 1, g0 + 1, g1 + 1, dx + 1, gr + 1)}


HARNESS_HEAD = r'''// GENERATED by oracle/ref_extract.py from /root/reference (test infrastructure).
#include <algorithm>
#include <cmath>
#include <cstring>
'''


def write_source(path):
    defs, solve, fit_body, params, where = extract()
    src = [HARNESS_HEAD]
    src += defs
    src.append("namespace surfref {")
    src.append(f"// surfd.cu:{where[0]}")
    src += solve
    src.append("struct ref_dims { int x, y, z; };")
    src.append(f"// surfd.cu:{where[1]} (body)")
    src.append("float hFitQuadrat(float* src, float* _offsets, ref_dims* swhps, int* params, const int s, "
               "const int r, const int c, const int o)")
    src += fit_body
    src.append(f"// surfd.cu:{where[2]}-{where[3]}")
    src.append("void hessian_params(ref_dims swhp, int init_scale, int max_scale, int& init_mask_size, "
               "int init_border, int* borders, int octave, int sampling, int* params_out, float* norms_out)")
    src.append("{")
    src += params
    src.append("\tstd::memcpy(params_out, params, sizeof(params));")
    src.append("\tstd::memcpy(norms_out, norms, sizeof(norms));")
    src.append("\t(void)maxw; (void)maxh;")
    src.append("}")
    host = extract_host()
    w = host["where"]
    src.append("struct ref_its { int init_lobe; int sampling; };")
    src.append(f"// surf.cpp:{w[0]}, {w[1]} (initLut's loops)")
    src.append("void init_lut(float* table1, float* table2)")
    src.append("{")
    src += host["loop1"]
    src += host["loop2"]
    src.append("}")
    src.append(f"// surf.cpp:{w[2]}, {w[3]}, {w[4]} in the order of surf.cpp:241-293")
    src.append("void octave_plan(ref_its its, int noctaves, int max_scale, const int* swx, const int* swy, "
               "int* borders_out, int* params_out, float* norms_out)")
    src.append("{")
    src.append(host["mask"])
    src.append("\tint s = 0, octave = 1;")
    src.append("\tint border1 = 0;")
    src.append("\tint borders[MAX_OCTAVE] = {0};")
    src.append("\tfor (int o = 0; o < noctaves; o++)")
    src.append("\t{")
    src.append("\t\tif (o > 0)")
    src.append("\t\t{")
    src.append(host["border_o"])
    src.append("\t\t\tborders[0] = border1;")
    src.append("\t\t\tborders[1] = border1;")
    src.append("\t\t\ts = 2;")
    src.append("\t\t}")
    src.append("\t\telse")
    src.append("\t\t{")
    src.append(host["border_0"])
    src.append("\t\t}")
    src.append("\t\tref_dims d = {swx[o], swy[o], 0};")
    src.append("\t\thessian_params(d, s, max_scale, mask_size, border1, borders, octave, its.sampling, "
               "params_out + o * 7 * MAX_SCALE, norms_out + o * MAX_SCALE);")
    src.append("\t\tstd::memcpy(borders_out + o * MAX_OCTAVE, borders, sizeof(borders));")
    src.append("\t\toctave += octave;")
    src.append("\t}")
    src.append("}")
    more = extract_more()
    w2 = more["where"]
    src.append(f"// cuda_utils.h:{w2[0]}")
    src += more["align"]
    src.append("struct ref_param { bool doubled; int noctaves; float divisor; int init_lobe; int max_scale; "
               "int sampling; float thresh; bool upright; bool extend; int desc_wsz; int mag_factor; "
               "int orient_size; int nfeatures; };")
    src.append(f"// surf.cpp:{w2[1]}-{w2[2]} (Surfor::init)")
    src.append("void surfor_init(ref_param& its, ref_dims& whp, const int _noctaves, const float _thresh, "
               "const bool _doubled, const int _init_mask_size, const int _sampling_step, const bool _upright, "
               "const bool _extend, const int _desc_wsz, const int _width, const int _height)")
    src.append("{")
    src += more["init"]
    src.append("}")
    src.append(f"// surf.cpp:{w2[3]}-{w2[4]} (allocMemory's geometry)")
    src.append("int alloc_geometry(const ref_param& its, const int w, const int h, ref_dims& iwhp, ref_dims* swhps, "
               "int* osizes)")
    src.append("{")
    src += more["geo"]
    src.append("\treturn tot_osize;")
    src.append("}")
    src.append(f"// surfd.cu:{w2[5]}-{w2[6]} (cuFindMaximumWithInterp: NMS borders and grid)")
    src.append("void nms_grid(const ref_param& its, const int* borders, ref_dims whp, int* mborders_out, int* grid_out)")
    src.append("{")
    src += more["nms"]
    for k, e in enumerate(more["grid"]):
        src.append(f"\tgrid_out[{k}] = {e};")
    src.append("\tstd::memcpy(mborders_out, mborders, sizeof(mborders));")
    src.append("\t(void)b;")
    src.append("#undef DX")
    src.append("#undef DY")
    src.append("}")
    src.append("}  // namespace surfref")
    src.append(r'''
extern "C" {
int ref_max_scale(void) { return MAX_SCALE; }
int ref_max_octave(void) { return MAX_OCTAVE; }
void ref_solve(float* sol, float* sq9)
{
    float m[3][3];
    for (int i = 0; i < 9; i++) m[i / 3][i % 3] = sq9[i];
    surfref::hSolveLinearSystem(sol, m, 3);
    for (int i = 0; i < 9; i++) sq9[i] = m[i / 3][i % 3];
}
// one octave (o = 0) whose scale planes sit at src, plane size osize, row pitch sp
float ref_fit(float* src, float* off, int s, int r, int c, int osize, int sp)
{
    surfref::ref_dims swhps[MAX_OCTAVE] = {};
    swhps[0].z = sp;
    int params[3 * MAX_OCTAVE] = {0};
    params[MAX_OCTAVE + 0] = osize;          // osizes[o]
    params[2 * MAX_OCTAVE + 0] = 0;          // offsets[o]
    return surfref::hFitQuadrat(src, off, swhps, params, s, r, c, 0);
}
void ref_init_lut(float* t1, float* t2) { surfref::init_lut(t1, t2); }
// Surfor::detectAndCompute's octave loop (borders before each octave's NMS,
// every octave's Hessian parameters): borders [noct][MAX_OCTAVE], params
// [noct][7 MAX_SCALE], norms [noct][MAX_SCALE]
void ref_octave_plan(int init_lobe, int sampling, int noctaves, int max_scale, const int* swx, const int* swy,
                     int* borders, int* params, float* norms)
{
    surfref::ref_its its = {init_lobe, sampling};
    surfref::octave_plan(its, noctaves, max_scale, swx, swy, borders, params, norms);
}
// Surfor::init: out = {doubled, noctaves, divisor (bits), init_lobe, max_scale,
// sampling, thresh (bits), upright, extend, desc_wsz, mag_factor, orient_size,
// nfeatures, whp.x, whp.y, whp.z}
void ref_surfor_init(int* out, int noctaves, float thresh, int doubled, int init_mask_size, int sampling_step,
                     int upright, int extend, int desc_wsz, int width, int height)
{
    surfref::ref_param its = {};
    surfref::ref_dims whp = {};
    surfref::surfor_init(its, whp, noctaves, thresh, doubled != 0, init_mask_size, sampling_step, upright != 0,
                         extend != 0, desc_wsz, width, height);
    int v[16] = {its.doubled, its.noctaves, 0, its.init_lobe, its.max_scale, its.sampling, 0, its.upright,
                 its.extend, its.desc_wsz, its.mag_factor, its.orient_size, its.nfeatures, whp.x, whp.y, whp.z};
    std::memcpy(&v[2], &its.divisor, 4);
    std::memcpy(&v[6], &its.thresh, 4);
    std::memcpy(out, v, sizeof(v));
}
// allocMemory's geometry: iwhp[3], swhps[3 * MAX_OCTAVE], osizes[MAX_OCTAVE]; returns tot_osize
int ref_alloc_geometry(int doubled, int sampling, int max_scale, int noctaves, int w, int h, int* iwhp3,
                       int* swhps3, int* osizes)
{
    surfref::ref_param its = {};
    its.doubled = doubled != 0;
    its.sampling = sampling;
    its.max_scale = max_scale;
    its.noctaves = noctaves;
    surfref::ref_dims iwhp = {}, swhps[MAX_OCTAVE] = {};
    const int tot = surfref::alloc_geometry(its, w, h, iwhp, swhps, osizes);
    iwhp3[0] = iwhp.x; iwhp3[1] = iwhp.y; iwhp3[2] = iwhp.z;
    for (int o = 0; o < MAX_OCTAVE; o++) {
        swhps3[3 * o] = swhps[o].x; swhps3[3 * o + 1] = swhps[o].y; swhps3[3 * o + 2] = swhps[o].z;
    }
    return tot;
}
// NMS borders and grid extent of one octave (grid in blocks of DX x DY threads)
void ref_nms_grid(int max_scale, const int* borders, int swx, int swy, int* mborders, int* grid3)
{
    surfref::ref_param its = {};
    its.max_scale = max_scale;
    surfref::ref_dims whp = {swx, swy, 0};
    surfref::nms_grid(its, borders, whp, mborders, grid3);
}
void ref_hessian_params(int swx, int swy, int init_scale, int max_scale, int* init_mask_size, int init_border,
                        int* borders, int octave, int sampling, int* params_out, float* norms_out)
{
    surfref::ref_dims d = {swx, swy, 0};
    surfref::hessian_params(d, init_scale, max_scale, *init_mask_size, init_border, borders, octave, sampling,
                            params_out, norms_out);
}
}
''')
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as fh:
        fh.write("\n".join(src) + "\n")


def build():
    if not os.path.exists(os.path.join(REF, "surfd.cu")):
        print("ref_extract: no reference sources; oracle/_ref not built")
        return None
    cpp = os.path.join(OUT, "ref_host.cpp")
    so = os.path.join(OUT, "libref_host.so")
    write_source(cpp)
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
                           "-Wall", "-o", so, cpp])
    return so


if __name__ == "__main__":
    so = build()
    print(so or "skipped")
    sys.exit(0)
