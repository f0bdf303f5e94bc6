#!/usr/bin/env python3
"""Generate cuda-surf_amd/csrc/surfhip_far.inc: the unrolled corner programs
of the far-octave Hessian kernel (k_hess_far, octaves 2..4 of the default
geometry: init_lobe 3, sampling 2).

The reference's getHessian (surfd.cu:353-366) reads 32 integral-image
corners per scale through getSum (surfd.cu:334-343).  For a response sample
(y0, x0) = (delta*iy, delta*ix) every corner is I(y0 + dr, x0 + dc) with a
weight (+-1 for the outer / quadrant boxes, -+3 for the inner boxes) and a
sum it belongs to (dxx, dyy, dxy of one scale = slot 0..8).  Corners are
grouped by (dr, slot) and bucketed by rho = dr mod delta: integral row Y
contributes exactly the groups of class Y mod delta, to sample row
iy = (Y - dr) / delta.

The corner groups of a step's rows are dealt to the workgroup's waves by
cost (emit_balanced); each wave reads its groups' corners from the
residue-plane LDS ring (plane = column mod 8, so lane j's corner is a
compile-time offset from the lane's base) and adds each group's weighted
sum into its LDS accumulator.  Programs are emitted for 8- and 16-row steps
(SURF_FAR_R selects one at compile time).
"""
import os
import sys

VARIANTS = {            # octave: (delta, lobes of the three computed scales)
    2: (8, (31, 39, 47)),
    3: (16, (63, 79, 95)),
    4: (32, (127, 159, 191)),
}


def mulk(w, v):
    """w * v mod 2^32; 3 v as one full-rate v_lshl_add_u32 (mul3), since
    LLVM selects the quarter-rate v_mad_u64_u32 / v_mul_lo_u32 for 3u * v."""
    return f"mul3({v})" if w == 3 else f"{w}u * {v}"


def corners(m):
    x2 = m // 2
    x3, x4 = 2 * x2, 3 * x2
    out = []

    def box(x1, y1, xa, ya, w, slot):          # getSum(x1, y1, x2, y2), surfd.cu:334-343
        out.extend([(y1 + 1, x1 + 1, w, slot), (ya, xa, w, slot), (ya, x1 + 1, -w, slot), (y1 + 1, xa, -w, slot)])

    box(m + x2, x3, -m - x2, -x3, 1, 0)
    box(x2, x3, -x2, -x3, -3, 0)
    box(x3, m + x2, -x3, -m - x2, 1, 1)
    box(x3, x2, -x3, -x2, -3, 1)
    box(x4, 0, 0, -x4, 1, 2)
    box(0, x4, -x4, 0, 1, 2)
    box(x4, x4, 0, 0, -1, 2)
    box(0, 0, -x4, -x4, -1, 2)
    return out


def groups(oct_):
    d, lobes = VARIANTS[oct_]
    acc = {}
    for i, m in enumerate(lobes):
        for dr, dc, w, s in corners(m):
            key = (dr, 3 * i + s)
            acc.setdefault(key, {})
            acc[key][dc] = acc[key].get(dc, 0) + w
    out = {}
    for (dr, slot), cs in sorted(acc.items()):
        cs = [(dc, w) for dc, w in sorted(cs.items()) if w != 0]
        if cs:
            out.setdefault(dr % d, []).append((dr, slot, cs))
    return d, out


OCTS = (2, 3, 4)
RS = (8, 16)            # rows per step (= waves per workgroup) variants, selected by SURF_FAR_R


def emit_balanced(R):
    """Per-wave programs for steps of R integral rows (one ring row per wave):
    a step carries, per far octave of delta d, the corner groups of the
    residues (R ph + j) mod d of its rows j (ph: the step's phase when d > R).
    Every (octave, row, group) item of a step phase is dealt to the R waves
    by cost (greedy, largest first: residue costs differ up to 9x, so a
    wave-per-row split waited on the busiest row); each wave reads its items'
    rows from the ring and adds into the LDS accumulators (ds_add, so waves
    may share one).  Sample row of an item: i + k with i = Y0 / d (floor) and
    k = ((R ph) mod d + j - dr) / d; accumulator row (i + k) mod NA, from
    b = i mod NA computed once per step (far_wrap)."""
    nw = R
    out = ["", f"// ---- load-balanced per-wave programs, {R} rows per step (see emit_balanced)"]
    for nfar in (1, 2, 3):
        dmax = VARIANTS[OCTS[nfar - 1]][0]
        nph = max(1, dmax // R)
        for ph in range(nph):
            items = []
            for oi in range(nfar):
                o = OCTS[oi]
                d, g = groups(o)
                off = (R * ph) % d
                for j in range(R):
                    rho = (off + j) % d
                    for (dr, slot, cs) in g.get(rho, []):
                        k = (off + j - dr) // d
                        assert (off + j - dr) % d == 0
                        items.append((len(cs) + 1, oi, d, j, k, dr, slot, cs))
            items.sort(key=lambda t: (-t[0], t[1], t[3], t[5], t[6]))
            load = [0] * nw
            bins = [[] for _ in range(nw)]
            for it in items:
                w = min(range(nw), key=lambda i: (load[i], i))
                load[w] += it[0]
                bins[w].append(it)
            out.append(f"// nfar {nfar} phase {ph}: wave loads {load}")
            for w in range(nw):
                out.append("template <int H, int PL, int ROWW, int ST>")
                out.append(f"__device__ __forceinline__ void far_bal_n{nfar}_p{ph}_w{w}(const uint32_t* __restrict__ ring, "
                           "int lane, int* __restrict__ a0, int* __restrict__ a1, int* __restrict__ a2, int i0, int i1, "
                           "int i2, int s0, int s1, int s2, int b0, int b1, int b2)")
                out.append("{")
                for oi in range(nfar):
                    mine = [it for it in bins[w] if it[1] == oi]
                    if not mine:
                        continue
                    d = mine[0][2]
                    ls = d // 8
                    out.append(f"    if (lane < ST / {d}) {{")
                    out.append(f"        const uint32_t* rb = ring + {ls} * lane;")
                    for n, (_, _, _, j, k, dr, slot, cs) in enumerate(mine):
                        terms = []
                        for dc, wt in cs:
                            v = f"rb[{j} * ROWW + ((H + ({dc})) & 7) * PL + ((H + ({dc})) >> 3)]"
                            if wt == 1:
                                terms.append(f"+ {v}")
                            elif wt == -1:
                                terms.append(f"- {v}")
                            elif wt > 0:
                                terms.append(f"+ {mulk(wt, v)}")
                            else:
                                terms.append(f"- {mulk(-wt, v)}")
                        expr = " ".join(terms)
                        expr = expr[2:] if expr.startswith("+ ") else "0u " + expr
                        out.append(f"        const uint32_t t{n} = {expr};")
                    for n, (_, _, _, j, k, dr, slot, cs) in enumerate(mine):
                        out.append(f"        if ((unsigned)(i{oi} + ({k})) < (unsigned)s{oi})")
                        out.append(f"            atomicAdd(a{oi} + (far_wrap<{k}>(b{oi}) * 9 + {slot}) * "
                                   f"(ST / {d}), (int)t{n});")
                    out.append("    }")
                out.append("}")
                out.append("")
    # dispatcher: step index Y0 / R gives the phase
    out.append("template <int H, int PL, int ROWW, int ST>")
    out.append("__device__ __forceinline__ void far_bal(int nfar, int step, int w, const uint32_t* __restrict__ ring, "
               "int lane, int* a0, int* a1, int* a2, int i0, int i1, int i2, int s0, int s1, int s2, int b0, int b1, "
               "int b2)")
    out.append("{")
    out.append(f"    const int ph = step & ((nfar == 3 ? {max(1, 32 // R)} : nfar == 2 ? {max(1, 16 // R)} : 1) - 1);")
    out.append(f"    switch (((nfar - 1) * 4 + ph) * {nw} + w) {{")
    for nfar in (1, 2, 3):
        dmax = VARIANTS[OCTS[nfar - 1]][0]
        for ph in range(max(1, dmax // R)):
            for w in range(nw):
                out.append(f"    case {((nfar - 1) * 4 + ph) * nw + w}: far_bal_n{nfar}_p{ph}_w{w}<H, PL, ROWW, ST>(ring, lane, "
                           "a0, a1, a2, i0, i1, i2, s0, s1, s2, b0, b1, b2); break;")
    out.append("    default: break;")
    out.append("    }")
    out.append("}")
    out.append("")
    return out


def emit():
    lines = ["// Generated by tools/gen_far.py -- do not edit.",
             "// Far-octave corner programs for k_hess_far (see the generator's docstring).",
             "",
             "// accumulator row (i + K) mod NA from b = i mod NA (the row index of a",
             "// valid sample row i + K >= 0; |K| < NA): one conditional wrap",
             "template <int K>",
             "__device__ __forceinline__ int far_wrap(int b)",
             "{",
             "    const int t = b + K;",
             "    if constexpr (K >= 0) return t >= farc::NA ? t - farc::NA : t;",
             "    else return t < 0 ? t + farc::NA : t;",
             "}",
             ""]
    for i, R in enumerate(RS):
        lines.append(("#if" if i == 0 else "#elif") + f" SURF_FAR_R == {R}")
        lines.extend(emit_balanced(R))
    lines.append("#else")
    lines.append("#error \"SURF_FAR_R: no corner programs generated for this step height\"")
    lines.append("#endif")
    return "\n".join(lines) + "\n"


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "cuda-surf_amd",
                                                             "csrc", "surfhip_far.inc")
    with open(out, "w") as fh:
        fh.write(emit())
    print("wrote", out)
