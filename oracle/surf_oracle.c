/*
 * surf_oracle.c -- scalar CPU restatement of the CUDA-SURF hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see surf_oracle.h): the parity checker and the
 * CPU baseline.  Build with -ffp-contract=off; every float expression below
 * is written in the reference's evaluation order, one IEEE rounding per
 * operation, and double-precision M_PI terms are kept where the reference
 * mixes `M_PI` (a double) into float expressions.
 *
 * Parity status: "parity unpinned" vs the CUDA binary (cannot be built or
 * run here, and the reference holds no golden outputs) -- see header.
 */
#define _GNU_SOURCE
#include "surf_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

_Static_assert(sizeof(or_point) == 48, "SurfPoint must stay 48 bytes");
_Static_assert(sizeof(or_param) == 48, "SurfParam must stay 48 bytes");

/* surfd.h:148-155 */
#define NBIN       72
#define WINDOW     1.0471975511965976f   /* M_PI / 3         */
#define SEP_ANGLE  0.08726646259971647f  /* 2 * M_PI / NBIN  */
#define HWN        6
#define ORADIUS    9
#define ORADIUSSQ  81.5f
#define H_PI       1.5707963267948966f   /* cuda_utils.h:8   */
#define INV255     0.003921568627f       /* surfd.cu:356     */

static inline int align_up(int a, int b) { return (a % b != 0) ? (a - a % b + b) : a; } /* cuda_utils.h:160-163 */
static inline int f2i_rn(float v) { return (int)rintf(v); }   /* __float2int_rn */
static inline int f2i_rz(float v) { return (int)v; }          /* __float2int_rz */

/* ------------------------------------------------------------------ init */

/* surf.cpp:60-91 */
int or_init_param(or_param* p, int noctaves, float thresh, bool doubled,
                  int init_mask_size, int sampling_step, bool upright,
                  bool extend, int desc_wsz)
{
    memset(p, 0, sizeof(*p));
    if (noctaves < 1 || noctaves > OR_MAX_OCTAVE) return -1;
    /* desc_wsz <= 7: a sample's Gaussian weight is lookup2[(int)(rpos^2 +
     * cpos^2)] (surfd.cu:1303, 1335, 1999) with |rpos|, |cpos| <
     * (desc_wsz + 1) / 2, and lookup2 has 40 entries (surfd.cu:23): from
     * desc_wsz 8 on the reference reads past it */
    if (desc_wsz < 1 || desc_wsz > 7) return -1;
    p->doubled = doubled;
    p->noctaves = noctaves;
    p->divisor = doubled ? 0.5f : 1.f;
    p->init_lobe = init_mask_size / 3;
    p->max_scale = p->init_lobe + 2;
    p->sampling = sampling_step + (doubled ? sampling_step : 0);
    p->thresh = thresh;
    p->upright = upright;
    p->extend = extend;
    p->desc_wsz = desc_wsz;
    p->mag_factor = 12 / desc_wsz;
    p->orient_size = 4 + (extend ? 4 : 0);
    p->nfeatures = desc_wsz * desc_wsz * p->orient_size;
    /* scales per octave: MAX_SCALE bounds them (surfd.h:9); below 4 the
     * octaves > 0 compute fewer than 2 scales and the lobes degenerate */
    if (p->max_scale < 4 || p->max_scale > OR_MAX_SCALE) return -1;
    return 0;
}

/* surf.cpp:358-371 (LUTs) and surf.cpp:83-89 (bins, float accumulation from
 * (float)-CV_PI). */
void or_init_tables(float lut1[83], float lut2[40], float bins[OR_NBIN])
{
    for (int n = 0; n < 83; n++) lut1[n] = expf(-(n + 0.5f) / 12.5f);
    for (int n = 0; n < 40; n++) lut2[n] = expf(-(n + 0.5f) / 8.f);
    bins[0] = (float)(-M_PI);
    for (int i = 1; i < NBIN; i++) bins[i] = bins[i - 1] + SEP_ANGLE;
}

/* surf.cpp:374-392 */
void or_geometry(const or_param* p, int w, int h, or_geom* g)
{
    memset(g, 0, sizeof(*g));
    g->iwhp.x = p->doubled ? w + w - 1 : w + 1;       /* surf.cpp:377-378 */
    g->iwhp.y = p->doubled ? h + h - 1 : h + 1;
    g->iwhp.z = align_up(g->iwhp.x, 128);
    g->swhp[0].x = (g->iwhp.x - 1) / p->sampling;
    g->swhp[0].y = (g->iwhp.y - 1) / p->sampling;
    g->swhp[0].z = align_up(g->swhp[0].x, 128);
    g->osize[0] = g->swhp[0].y * g->swhp[0].z;
    size_t off = 0;
    g->ooff[0] = 0;
    off += (size_t)g->osize[0] * p->max_scale;
    for (int j = 1; j < p->noctaves; j++) {
        g->swhp[j].x = g->swhp[j - 1].x >> 1;
        g->swhp[j].y = g->swhp[j - 1].y >> 1;
        g->swhp[j].z = align_up(g->swhp[j].x, 128);
        g->osize[j] = g->swhp[j].y * g->swhp[j].z;
        g->ooff[j] = off;
        off += (size_t)g->osize[j] * p->max_scale;
    }
    g->tot_osize = off;
}

/* Host recurrences: surf.cpp:240-292 (mask_size, border1, borders[0..1]),
 * surfd.cu:2844-2865 (per-scale Hessian params, borders[s] = value BEFORE the
 * s>2 update), surfd.cu:3062-3076 (NMS borders and launch extent). */
void or_octave_params(const or_param* p, const or_geom* g, or_octave oct[OR_MAX_OCTAVE])
{
    int mask_size = p->init_lobe - 2;            /* surf.cpp:240 */
    int octave = 1;
    int borders[OR_MAX_SCALE] = {0};
    for (int o = 0; o < p->noctaves; o++) {
        or_octave* q = &oct[o];
        memset(q, 0, sizeof(*q));
        int s, border1;
        if (o > 0) {                              /* surf.cpp:250-265 */
            border1 = ((3 * (mask_size + 4 * octave)) / 2) / (p->sampling * octave) + 1;
            borders[0] = border1;
            borders[1] = border1;
            s = 2;
        } else {                                  /* surf.cpp:266-270 */
            border1 = ((3 * (mask_size + 6 * octave)) / 2) / (p->sampling * octave) + 1;
            s = 0;
        }
        q->octave = octave;
        q->init_scale = s;
        q->nscale = p->max_scale - s;
        q->delta = p->sampling * octave;
        /* cuCalcHessianMulti, surfd.cu:2844-2865 */
        for (int i = 0, ss = s; ss < p->max_scale; i++, ss++) {
            borders[ss] = border1;
            int m = mask_size + 2 * octave * (i + 1);
            if (ss > 2) border1 = 3 * m / 2 / q->delta + 1;
            q->mask[i] = m;
            q->border1[i] = border1;
            float nrm = 9.f / (float)(m * m);
            nrm *= nrm;
            q->norm[i] = nrm;
            q->x2[i] = m / 2;
            q->x3[i] = q->x2[i] + q->x2[i];
            q->x4[i] = q->x2[i] + q->x3[i];
        }
        mask_size = q->mask[q->nscale - 1];       /* surfd.cu:2865 */
        for (int k = 0; k < OR_MAX_SCALE; k++) q->borders[k] = borders[k];
        /* cuFindMaximumWithInterp, surfd.cu:3062-3076 */
        int n = 0, maxw = 0, maxh = 0;
        for (int k = 1; k < p->max_scale - 1; k += 2) {
            q->mborders[n] = borders[k + 1] + 1;
            int b = q->mborders[n] + q->mborders[n];
            if (g->swhp[o].x - b > maxw) maxw = g->swhp[o].x - b;
            if (g->swhp[o].y - b > maxh) maxh = g->swhp[o].y - b;
            n++;
        }
        q->nms_gx = ((maxw / 2 + 16 - 1) / 16) * 16;
        q->nms_gy = ((maxh / 2 + 16 - 1) / 16) * 16;
        octave += octave;                         /* surf.cpp:293 */
    }
}

/* -------------------------------------------------------------- integral */

/* integralRow / integralCol (surfd.cu:129-165).  ii[(y+1)*p + x+1] holds the
 * sum of img over rows <= y, cols <= x.  Row 0 and column 0 are written as 0
 * (fixed semantics).  Arithmetic in uint32 (wraparound). */
void or_integral(const uint8_t* img, int w, int h, int pitch, int32_t* ii, int ipitch)
{
    for (int x = 0; x <= w; x++) ii[x] = 0;
    for (int y = 0; y < h; y++) {
        uint32_t* dst = (uint32_t*)ii + (size_t)(y + 1) * ipitch;
        const uint32_t* up = (const uint32_t*)ii + (size_t)y * ipitch;
        const uint8_t* src = img + (size_t)y * pitch;
        uint32_t row = 0;
        dst[0] = 0;
        for (int x = 0; x < w; x++) {
            row += src[x];
            dst[x + 1] = up[x + 1] + row;   /* column pass folded in */
        }
    }
}

/* Doubled image (cuIntegralDoubleU4, surfd.cu:2707-2772): the first kernel
 * (integralDoubleRow0U2, surfd.cu:166-209) writes, for source pixel (y, x),
 * integral rows 2y+1 / 2y+2 and columns 2x+1 / 2x+2 from the 2x upsampled
 * image D with
 *   D[2y][2x]     = s[y][x]
 *   D[2y][2x+1]   = rn((s[y][x] + s[y][x+1]) * 0.5f)
 *   D[2y+1][2x]   = rn((s[y][x] + s[y+1][x]) * 0.5f)
 *   D[2y+1][2x+1] = rn((s[y][x] + s[y][x+1] + s[y+1][x] + s[y+1][x+1]) * 0.25f)
 * (__float2int_rn: round half to even) as running sums inside groups of 4
 * columns; integralRow1U4/Row2U4 (surfd.cu:212-259) chain the groups into
 * a row prefix and integralCol0U4/Col1U4/Col2U4 (surfd.cu:262-318) do the
 * same down the columns.  Net: ii = the integral of D over the
 * (2w-1) x (2h-1) integral grid (surf.cpp:377-378), i.e. D is
 * (2w-2) x (2h-2) and never needs s outside the image (the reference's
 * writes to integral row 2h-1 / 2h and column 2w-1 / 2w, which read source
 * row h / column w, fall outside that grid and are dropped here). */
void or_double_image(const uint8_t* img, int w, int h, int pitch, uint8_t* dst, int dpitch)
{
    const int W2 = 2 * w - 2, H2 = 2 * h - 2;
    for (int r = 0; r < H2; r++) {
        const int y = r >> 1;
        const uint8_t* s0 = img + (size_t)y * pitch;
        const uint8_t* s1 = (r & 1) ? s0 + pitch : s0;
        for (int c = 0; c < W2; c++) {
            const int x = c >> 1;
            int v;
            if (!(r & 1) && !(c & 1)) v = s0[x];
            else if (!(r & 1)) v = (int)rintf((float)(s0[x] + s0[x + 1]) * 0.5f);
            else if (!(c & 1)) v = (int)rintf((float)(s0[x] + s1[x]) * 0.5f);
            else v = (int)rintf((float)(s0[x] + s0[x + 1] + s1[x] + s1[x + 1]) * 0.25f);
            dst[(size_t)r * dpitch + c] = (uint8_t)v;
        }
    }
}

/* --------------------------------------------------------------- Hessian */

/* getSum (surfd.cu:334-343): sum of the inclusive rect [x2..x1] x [y2..y1]. */
static inline uint32_t box(const int32_t* d, int x1, int y1, int x2, int y2, int p)
{
    const uint32_t* u = (const uint32_t*)d;
    long yp1 = (long)y1 * p + p;
    long yp2 = (long)y2 * p;
    return u[yp1 + x1 + 1] + u[yp2 + x2] - u[yp2 + x1 + 1] - u[yp1 + x2];
}

/* getHessian (surfd.cu:353-366); v = vas[0..8] as built in surfd.cu:466-477. */
static float hessian_at(const int32_t* d, const int* v, int p)
{
    const float r = INV255;
    const float rr = r * r;
    const int32_t sxx = (int32_t)(box(d, v[5] + v[2], v[1] + v[3], v[6] - v[2], v[1] - v[3], p)
                                  - 3u * box(d, v[0] + v[2], v[1] + v[3], v[0] - v[2], v[1] - v[3], p));
    const int32_t syy = (int32_t)(box(d, v[0] + v[3], v[7] + v[2], v[0] - v[3], v[8] - v[2], p)
                                  - 3u * box(d, v[0] + v[3], v[1] + v[2], v[0] - v[3], v[1] - v[2], p));
    const int32_t sxy = (int32_t)(box(d, v[0] + v[4], v[1], v[0], v[1] - v[4], p)
                                  + box(d, v[0], v[1] + v[4], v[0] - v[4], v[1], p)
                                  - box(d, v[0] + v[4], v[1] + v[4], v[0], v[1], p)
                                  - box(d, v[0], v[1], v[0] - v[4], v[1] - v[4], p));
    const float dxx = (float)sxx;
    const float dyy = (float)syy;
    const float dxy = 0.6f * (float)sxy;
    const float a = dxx * dyy;
    const float b = dxy * dxy;
    return rr * (a - b);
}

/* getSum for getTrace: makePoint builds its box from the interpolated scale
 * (surfd.cu:1010-1020) without a bounds check, so near the image border a
 * corner can fall outside [0, W] x [0, H] (e.g. column -1).  The reference
 * then reads the flat pitched buffer at that index: column -1 of row y is
 * the zero pad at the end of row y-1.  This restates that flat read, with
 * zero pad columns, and defines reads outside the frame's buffer as 0. */
static inline uint32_t flat_at(const uint32_t* u, long idx, long len)
{
    return (idx >= 0 && idx < len) ? u[idx] : 0u;
}
static inline uint32_t box_flat(const int32_t* d, int x1, int y1, int x2, int y2, int p, long len)
{
    const uint32_t* u = (const uint32_t*)d;
    long yp1 = (long)y1 * p + p;
    long yp2 = (long)y2 * p;
    return flat_at(u, yp1 + x1 + 1, len) + flat_at(u, yp2 + x2, len) - flat_at(u, yp2 + x1 + 1, len) -
           flat_at(u, yp1 + x2, len);
}

/* getTrace (surfd.cu:369-377). */
static int trace_at(const int32_t* d, const int* v, int p, long len)
{
    const int32_t lxx = (int32_t)(box_flat(d, v[5] + v[2], v[1] + v[3], v[6] - v[2], v[1] - v[3], p, len)
                                  - 3u * box_flat(d, v[0] + v[2], v[1] + v[3], v[0] - v[2], v[1] - v[3], p, len));
    const int32_t lyy = (int32_t)(box_flat(d, v[0] + v[3], v[7] + v[2], v[0] - v[3], v[8] - v[2], p, len)
                                  - 3u * box_flat(d, v[0] + v[3], v[1] + v[2], v[0] - v[3], v[1] - v[2], p, len));
    return ((int32_t)((uint32_t)lxx + (uint32_t)lyy) > 0) ? 1 : -1;
}

/* halfImage (surfd.cu:321-331) + calcHessianMultiConst (surfd.cu:445-481)
 * driven as in surf.cpp:248-294.  Cells outside a scale's valid window are 0
 * (the reference gets them from cudaMemset, surf.cpp:348). */
void or_hessian(const or_param* p, const or_geom* g, const or_octave* oct,
                const int32_t* ii, float* resp)
{
    const int ip = g->iwhp.z;
    for (int o = 0; o < p->noctaves; o++) {
        const or_octave* q = &oct[o];
        const int sw = g->swhp[o].x, sh = g->swhp[o].y, sp = g->swhp[o].z;
        float* base = resp + g->ooff[o];
        if (o > 0) {
            /* dof0 <- sof0 (plane max_scale - 3 of o-1), dof1 <- sof1 (plane
             * max_scale - 1; surf.cpp:252-258: offset - 3 / - 1 planes) */
            const float* prev = resp + g->ooff[o - 1];
            const int pp = g->swhp[o - 1].z;
            const size_t pos = (size_t)g->osize[o - 1];
            for (int t = 0; t < 2; t++) {
                const float* src = prev + (size_t)(t == 0 ? p->max_scale - 3 : p->max_scale - 1) * pos;
                float* dst = base + (size_t)t * g->osize[o];
                memset(dst, 0, sizeof(float) * g->osize[o]);
                for (int iy = 0; iy < sh; iy++)
                    for (int ix = 0; ix < sw; ix++)
                        dst[(size_t)iy * sp + ix] = src[(size_t)2 * iy * pp + 2 * ix];
            }
        }
        for (int i = 0; i < q->nscale; i++) {
            const int s = q->init_scale + i;
            float* dst = base + (size_t)s * g->osize[o];
            memset(dst, 0, sizeof(float) * g->osize[o]);
            const int b1 = q->border1[i];
            if (sw - b1 > b1 && sh - b1 > b1) {
                /* every box corner must stay inside the integral image
                 * (the reference never checks) */
                const int reach = q->mask[i] + q->x2[i] > q->x4[i] ? q->mask[i] + q->x2[i] : q->x4[i];
                const int lo_x = q->delta * b1 - reach, hi_x = q->delta * (sw - b1 - 1) + reach + 1;
                const int lo_y = q->delta * b1 - reach, hi_y = q->delta * (sh - b1 - 1) + reach + 1;
                if (lo_x < 0 || lo_y < 0 || hi_x >= g->iwhp.x || hi_y >= g->iwhp.y) {
                    fprintf(stderr, "oracle: Hessian box out of range o=%d s=%d\n", o, s);
                    abort();
                }
            }
            for (int iy = b1; iy < sh - b1; iy++) {
                for (int ix = b1; ix < sw - b1; ix++) {
                    int v[9];
                    v[2] = q->x2[i];
                    v[3] = q->x3[i];
                    v[4] = q->x4[i];
                    v[1] = q->delta * iy;            /* border2 + delta * y */
                    v[7] = v[1] + q->mask[i];
                    v[8] = v[1] - q->mask[i];
                    v[0] = q->delta * ix;
                    v[5] = v[0] + q->mask[i];
                    v[6] = v[0] - q->mask[i];
                    const float hv = hessian_at(ii, v, ip);
                    dst[(size_t)iy * sp + ix] = hv * q->norm[i];
                }
            }
        }
    }
}

/* ---------------------------------------------------- NMS + interpolation */

/* solveLinearSystem (surfd.cu:835-887), including the reference's `pivot`
 * that is not reset between columns. */
static void solve3(float* sol, float sq[3][3])
{
    const int size = 3;
    int row, col, c, pivot = 0, i;
    float maxc, coef, temp, mult, val;
    for (col = 0; col < size - 1; col++) {
        maxc = -1.f;
        for (row = col; row < size; row++) {
            coef = sq[row][col];
            coef = (coef < 0.f ? -coef : coef);
            if (coef > maxc) { maxc = coef; pivot = row; }
        }
        if (pivot != col) {
            for (i = 0; i < size; i++) {
                temp = sq[pivot][i]; sq[pivot][i] = sq[col][i]; sq[col][i] = temp;
            }
            temp = sol[pivot]; sol[pivot] = sol[col]; sol[col] = temp;
        }
        for (row = col + 1; row < size; row++) {
            mult = sq[row][col] / sq[col][col];
            for (c = col; c < size; c++) {
                const float t = mult * sq[col][c];
                sq[row][c] = sq[row][c] - t;
            }
            const float t = mult * sol[col];
            sol[row] = sol[row] - t;
        }
    }
    for (row = size - 1; row >= 0; row--) {
        val = sol[row];
        for (col = size - 1; col > row; col--) {
            const float t = sol[col] * sq[row][col];
            val = val - t;
        }
        sol[row] = val / sq[row][row];
    }
}

/* fitQuadrat (surfd.cu:942-988). */
static float fit_quadratic(const float* src, float off[3], int s, int r, int c, int osize, int sp)
{
    const float* cur = src + (size_t)s * osize;
    const float* prv = cur - osize;
    const float* nxt = cur + osize;
    const long idx = (long)r * sp + c;
    const long inr = idx + sp, ipr = idx - sp, inc = idx + 1, ipc = idx - 1;
    float g[3], H[3][3];
    g[0] = (nxt[idx] - prv[idx]) * 0.5f;
    g[1] = (cur[inr] - cur[ipr]) * 0.5f;
    g[2] = (cur[inc] - cur[ipc]) * 0.5f;
    const float temp = cur[idx] + cur[idx];
    H[0][0] = (prv[idx] + nxt[idx]) - temp;
    H[1][1] = (cur[inr] + cur[ipr]) - temp;
    H[2][2] = (cur[inc] + cur[ipc]) - temp;
    H[0][1] = ((nxt[inr] - nxt[ipr]) - (prv[inr] - prv[ipr])) * 0.25f;
    H[0][2] = ((nxt[inc] - nxt[ipc]) - (prv[inc] - prv[ipc])) * 0.25f;
    H[1][2] = ((cur[inr + 1] - cur[inr - 1]) - (cur[ipr + 1] - cur[ipr - 1])) * 0.25f;
    H[1][0] = H[0][1];
    H[2][0] = H[0][2];
    H[2][1] = H[1][2];
    off[0] = -g[0];
    off[1] = -g[1];
    off[2] = -g[2];
    solve3(off, H);
    const float a = off[0] * g[0];
    const float b = off[1] * g[1];
    const float cc = off[2] * g[2];
    const float dot = (a + b) + cc;
    const float half = 0.5f * dot;
    return cur[idx] + half;
}

/* Evaluate one NMS block (surfd.cu:678-832 for thread (x, y, z)); on success
 * fills *pt (makePoint, surfd.cu:1001-1022) and returns 1. */
static int nms_block(const or_param* p, const or_geom* g, const or_octave* q, int o,
                     const int32_t* ii, const float* src, int z, int x, int y, or_point* pt)
{
    const int sw = g->swhp[o].x, sh = g->swhp[o].y, sp = g->swhp[o].z;
    const int osize = g->osize[o];
    const int k = 2 * z + 1;
    if (k >= p->max_scale - 1) return 0;
    const int mb = q->mborders[z];
    const int i = mb + y * 2;
    const int j = mb + x * 2;
    if (i >= sh - mb || j >= sw - mb) return 0;

    int iw = i * sp + j, ix = iw + 1, iy = iw + sp, iz = iy + 1;
    const float* cs = src + (size_t)k * osize;
    int cas = 0;
    float best = cs[iw];
    if (cs[ix] > best) { best = cs[ix]; cas = 1; }
    if (cs[iy] > best) { best = cs[iy]; cas = 2; }
    if (cs[iz] > best) { best = cs[iz]; cas = 3; }
    cs += osize;
    if (cs[iw] > best) { best = cs[iw]; cas = 4; }
    if (cs[ix] > best) { best = cs[ix]; cas = 5; }
    if (cs[iy] > best) { best = cs[iy]; cas = 6; }
    if (cs[iz] > best) { best = cs[iz]; cas = 7; }
    if (best < p->thresh * 0.8f || (k + 1 == p->max_scale - 1 && cas > 3)) return 0;

    int s = k, r = i, c = j;
    int ds = -1, dr = -1, dc = -1;
    if (cas != 0) {
        if (cas == 1) { c = j + 1; dc = 1; }
        else if (cas == 2) { r = i + 1; dr = 1; }
        else if (cas == 3) { c = j + 1; r = i + 1; dc = 1; dr = 1; }
        else {
            s++; ds = 1;
            if (cas == 5) { c = j + 1; dc = 1; }
            else if (cas == 6) { r = i + 1; dr = 1; }
            else if (cas == 7) { c = j + 1; r = i + 1; dc = 1; dr = 1; }
        }
    }
    /* the 19 neighbours outside the 2x2x2 block (surfd.cu:757-792) */
    int ss = s + ds;
    cs = src + (size_t)ss * osize;
    iy = (r - dr) * sp + c; ix = iy - 1; iz = iy + 1;
    if (best < cs[ix] || best < cs[iy] || best < cs[iz]) return 0;
    iy += dr * sp; ix = iy - 1; iz = iy + 1;
    if (best < cs[ix] || best < cs[iy] || best < cs[iz]) return 0;
    iy += dr * sp; ix = iy - 1; iz = iy + 1;
    if (best < cs[ix] || best < cs[iy] || best < cs[iz]) return 0;
    cs = src + (size_t)s * osize;
    if (best < cs[ix] || best < cs[iy] || best < cs[iz]) return 0;
    iw = r * sp + c + dc;
    if (best < cs[iw]) return 0;
    iw -= dr * sp;
    if (best < cs[iw]) return 0;
    ss = s - ds;
    cs = src + (size_t)ss * osize;
    if (best < cs[ix] || best < cs[iy] || best < cs[iz] || best < cs[iw]) return 0;
    iw += dr * sp;
    if (best < cs[iw]) return 0;

    /* interpolation, surfd.cu:795-819 */
    float off[3] = {0.f, 0.f, 0.f};
    float strength = 0.f;
    int newr = r, newc = c;
    for (int mv = 0; mv < 5; mv++) {                 /* moves_remain = 5, surf.cpp:288 */
        r = newr; c = newc;
        strength = fit_quadratic(src, off, s, r, c, osize, sp);
        if (off[1] > 0.6f && r < sh - q->borders[s]) newr++;
        if (off[1] < -0.6f && r > q->borders[s]) newr--;
        if (off[2] > 0.6f && c < sw - q->borders[s]) newc++;
        if (off[2] < -0.6f && c > q->borders[s]) newc--;
        if (newr == r && newc == c) break;
    }
    if (isnan(off[0]) || isnan(off[1]) || isnan(off[2]) ||
        fabsf(off[0]) > 1.5f || fabsf(off[1]) > 1.5f || fabsf(off[2]) > 1.5f ||
        strength < p->thresh)
        return 0;

    /* surfd.cu:822-824 */
    const int octave = q->octave;
    const float t0 = (float)s + off[0];
    const float t1 = t0 * 2.f;
    const float t2 = t1 * (float)octave;
    const float ns = ((float)(p->init_lobe + (octave - 1) * p->max_scale) + t2) / 3.f;
    const float ny = (float)octave * ((float)r + off[1]);
    const float nx = (float)octave * ((float)c + off[2]);

    /* makePoint, surfd.cu:1001-1022 */
    const float temp_delta = (float)p->sampling * p->divisor;
    memset(pt, 0, sizeof(*pt));
    pt->match = -1;
    pt->x = nx * temp_delta;
    pt->y = ny * temp_delta;
    pt->scale = (1.2f * ns) * p->divisor;
    pt->strength = strength;
    pt->ori = 0.f;
    pt->o = o;
    int v[9];
    const int temp = f2i_rz(fmaf(3.f, ns, 0.5f));
    v[0] = f2i_rz(fmaf(nx, (float)p->sampling, 0.5f));
    v[1] = f2i_rz(fmaf(ny, (float)p->sampling, 0.5f));
    v[2] = temp / 2;
    v[3] = v[2] + v[2];
    v[4] = v[2] + v[3];
    v[5] = v[0] + temp;
    v[6] = v[0] - temp;
    v[7] = v[1] + temp;
    v[8] = v[1] - temp;
    pt->laplace = trace_at(ii, v, g->iwhp.z, (long)g->iwhp.y * g->iwhp.z);
    return 1;
}

int or_find_points(const or_param* p, const or_geom* g, const or_octave* oct,
                   const int32_t* ii, const float* resp, or_point* pts, int max_pts)
{
    int count = 0;
    for (int o = 0; o < p->noctaves; o++) {
        const or_octave* q = &oct[o];
        const float* src = resp + g->ooff[o];
        /* grid z = the NMS levels k = 1, 3, .. < max_scale - 1 (surfd.cu:3064-3071) */
        for (int z = 0; z < (p->max_scale - 1) / 2; z++)
            for (int y = 0; y < q->nms_gy; y++)
                for (int x = 0; x < q->nms_gx; x++) {
                    or_point pt;
                    if (nms_block(p, g, q, o, ii, src, z, x, y, &pt)) {
                        if (count < max_pts) pts[count] = pt;
                        count++;
                    }
                }
    }
    return count;
}

/* ---------------------------------------------------------- descriptors */

/* getWavelet1 / getWavelet2 (surfd.cu:1171-1182). */
static inline int32_t wavelet1(const int32_t* d, int x, int y, int size, int p)
{
    return (int32_t)(box(d, x + size, y, x - size, y - size, p) -
                     box(d, x + size, y + size, x - size, y, p));
}
static inline int32_t wavelet2(const int32_t* d, int x, int y, int size, int p)
{
    return (int32_t)(box(d, x + size, y + size, x, y - size, p) -
                     box(d, x, y + size, x - size, y - size, p));
}

/* dFastAtan2 (surfd.cu:114-126); `M_PI - r` is evaluated in double. */
float or_fast_atan2(float y, float x)
{
    const float absx = fabsf(x);
    const float absy = fabsf(y);
    const float a = fminf(absx, absy) / fmaxf(absx, absy);
    const float s = a * a;
    float r = fmaf(fmaf(fmaf(-0.0464964749f, s, 0.15931422f), s, -0.327622764f), s * a, a);
    r = (absy > absx ? H_PI - r : r);
    r = (x < 0 ? (float)(M_PI - (double)r) : r);
    r = (y < 0 ? -r : r);
    return r;
}

/* Deterministic replacement for __sinf/__cosf (surfd.cu:2423-2424): Cody-Waite
 * reduction by pi/2 and Cephes single-precision polynomials, plain float ops
 * only (the HIP kernel evaluates the identical sequence). */
static float sincos_poly(float x, int want_cos)
{
    const float q = x * 0.636619772f;                 /* 2/pi */
    const float kf = rintf(q);
    int k = (int)kf;
    const float a = kf * 1.5703125f;                  /* pi/2 = C1 + C2 + C3 */
    const float b = kf * 4.837512969970703125e-4f;
    const float c = kf * 7.54978995489188216e-8f;
    const float r = ((x - a) - b) - c;
    const float z = r * r;
    /* sin(r) */
    float ps = -1.9515295891e-4f * z;
    ps = ps + 8.3321608736e-3f;
    ps = ps * z;
    ps = ps - 1.6666654611e-1f;
    ps = ps * z;
    ps = ps * r;
    const float sn = ps + r;
    /* cos(r) */
    float pc = 2.443315711809948e-5f * z;
    pc = pc - 1.388731625493765e-3f;
    pc = pc * z;
    pc = pc + 4.166664568298827e-2f;
    pc = pc * z;
    pc = pc * z;
    const float hz = 0.5f * z;
    const float cs = (pc - hz) + 1.0f;
    if (want_cos) k += 1;
    switch (k & 3) {
        case 0: return sn;
        case 1: return cs;
        case 2: return -sn;
        default: return -cs;
    }
}
float or_sinf(float x) { return sincos_poly(x, 0); }
float or_cosf(float x) { return sincos_poly(x, 1); }

/* assignOrientationApprox (surfd.cu:1711-1960).  Float sums accumulate in
 * row-major sample order (the reference's shared-memory atomics are
 * unordered); the window sums accumulate j = -6..6. */
float or_orientation(const or_param* p, const or_geom* g, const int32_t* ii,
                     const float lut1[83], const float bins[OR_NBIN], const or_point* pt)
{
    /* a doubled detector's integral is of the 2x frame: sample it at
     * (2x, 2y) with 2 * scale (surfd.cu:1734-1745) */
    const float scale = p->doubled ? pt->scale + pt->scale : pt->scale;
    const float x = p->doubled ? pt->x + pt->x : pt->x;
    const float y = p->doubled ? pt->y + pt->y : pt->y;
    const int pixsi = f2i_rz(2.f * scale + 1.6f);
    const int pixsi2 = f2i_rz(scale + 0.8f);
    const int ixo = f2i_rn(x), iyo = f2i_rn(y);
    int hist[NBIN];
    float avg[NBIN], part[NBIN], pas[NBIN + 2 * HWN], ws[NBIN], was[NBIN];
    memset(hist, 0, sizeof(hist));
    memset(avg, 0, sizeof(avg));
    memset(part, 0, sizeof(part));
    memset(pas, 0, sizeof(pas));
    memset(ws, 0, sizeof(ws));
    memset(was, 0, sizeof(was));
    const int ip = g->iwhp.z;
    for (int y1 = -ORADIUS; y1 <= ORADIUS; y1++) {
        for (int x1 = -ORADIUS; x1 <= ORADIUS; x1++) {
            const int xx = ixo + x1 * pixsi2;
            const int yy = iyo + y1 * pixsi2;
            if (!(yy + pixsi + 2 < g->iwhp.y && yy - pixsi > -1 &&
                  xx + pixsi + 2 < g->iwhp.x && xx - pixsi > -1)) continue;
            const int distsq = y1 * y1 + x1 * x1;
            if (!((float)distsq < ORADIUSSQ)) continue;
            const float dx = (float)wavelet2(ii, xx, yy, pixsi, ip) * INV255;
            const float dy = (float)wavelet1(ii, xx, yy, pixsi, ip) * INV255;
            const float m2 = dx * dx;
            const float n2 = dy * dy;
            const float mag = sqrtf(m2 + n2);
            if (!(mag > 0.f)) continue;
            const float weight = lut1[distsq];
            const float angle = or_fast_atan2(dy, dx);
            const int hid = f2i_rz((float)(((double)angle + M_PI) / (double)SEP_ANGLE)) % NBIN;
            const float psum = weight * mag;
            hist[hid] += 1;
            avg[hid] = avg[hid] + angle;
            part[hid] = part[hid] + psum;
            pas[hid + HWN] = pas[hid + HWN] + angle * psum;
            if (hid - HWN < 0)
                pas[hid + HWN + NBIN] = pas[hid + HWN + NBIN] + (float)(((double)angle + 2 * M_PI) * (double)psum);
            else if (hid + HWN >= NBIN)
                pas[hid + HWN - NBIN] = pas[hid + HWN - NBIN] + (float)(((double)angle - 2 * M_PI) * (double)psum);
        }
    }
    for (int t = 0; t < NBIN; t++)                   /* surfd.cu:1832-1835 */
        avg[t] = hist[t] > 0 ? avg[t] / (float)hist[t] : bins[t];

    for (int i = 0; i < NBIN; i++) {                 /* surfd.cu:1848-1908 */
        for (int j = -HWN; j <= HWN; j++) {
            int k = i + j;
            if (j == -HWN) {
                float residual;
                if (k < 0) {
                    k += NBIN;
                    const int k1 = (k + 1) % NBIN;
                    const float t = (bins[k1] + (WINDOW / 2)) - avg[i];
                    residual = (float)((double)t - (bins[k1] < 0 ? 0.0 : 2 * M_PI));
                } else {
                    residual = (bins[k + 1] + (WINDOW / 2)) - avg[i];
                }
                const float er = residual / SEP_ANGLE;
                ws[i] = ws[i] + er * part[k];
                was[i] = was[i] + er * pas[i];
            } else if (j == HWN) {
                float residual;
                if (k >= NBIN) {
                    k -= NBIN;
                    const float t = avg[i] + (WINDOW / 2);
                    residual = (float)(((double)t - 2 * M_PI) - (double)bins[k]);
                } else {
                    residual = (avg[i] + (WINDOW / 2)) - bins[k];
                }
                const float er = residual / SEP_ANGLE;
                ws[i] = ws[i] + er * part[k];
                was[i] = was[i] + er * pas[i + HWN + HWN];
            } else {
                was[i] = was[i] + pas[k + HWN];
                if (k < 0) k += NBIN;
                else if (k >= NBIN) k -= NBIN;
                ws[i] = ws[i] + part[k];
            }
        }
    }
    /* tree argmax, chunks of 64 then 8, strict '<' (surfd.cu:1921-1947) */
    for (int stride = 32; stride > 0; stride >>= 1)
        for (int t = 0; t < stride; t++)
            if (ws[t] < ws[t + stride]) { ws[t] = ws[t + stride]; was[t] = was[t + stride]; }
    for (int stride = 4; stride > 0; stride >>= 1)
        for (int t = 0; t < stride; t++)
            if (ws[64 + t] < ws[64 + t + stride]) { ws[64 + t] = ws[64 + t + stride]; was[64 + t] = was[64 + t + stride]; }
    if (ws[0] < ws[64]) { ws[0] = ws[64]; was[0] = was[64]; }
    return was[0] / ws[0];
}

/* placeInIndex (surfd.cu:1199-1271), accumulating in call order. */
static void place(float* desc, int wsz, int osz, float mag1, int ori1, float mag2, int ori2, float rx, float cx)
{
    const int ri = f2i_rz(rx >= 0.f ? rx : rx - 1.f);
    const int ci = f2i_rz(cx >= 0.f ? cx : cx - 1.f);
    const float rfrac = rx - (float)ri;
    const float cfrac = cx - (float)ci;
    const float cfrac1 = 1 - cfrac;
    int r_index = ri, c_index, ostart;
    float rw1, rw2, cw1, cw2;
    if (r_index >= 0) {
        rw1 = mag1 * (1.f - rfrac);
        rw2 = mag2 * (1.f - rfrac);
        c_index = ci;
        if (c_index >= 0) {
            cw1 = rw1 * cfrac1; cw2 = rw2 * cfrac1;
            ostart = r_index * wsz * osz + c_index * osz;
            desc[ostart + ori1] += cw1; desc[ostart + ori2] += cw2;
        }
        c_index++;
        if (c_index < wsz) {
            cw1 = rw1 * cfrac; cw2 = rw2 * cfrac;
            ostart = r_index * wsz * osz + c_index * osz;
            desc[ostart + ori1] += cw1; desc[ostart + ori2] += cw2;
        }
    }
    r_index++;
    if (r_index < wsz) {
        rw1 = mag1 * rfrac;
        rw2 = mag2 * rfrac;
        c_index = ci;
        if (c_index >= 0) {
            cw1 = rw1 * cfrac1; cw2 = rw2 * cfrac1;
            ostart = r_index * wsz * osz + c_index * osz;
            desc[ostart + ori1] += cw1; desc[ostart + ori2] += cw2;
        }
        c_index++;
        if (c_index < wsz) {
            cw1 = rw1 * cfrac; cw2 = rw2 * cfrac;
            ostart = r_index * wsz * osz + c_index * osz;
            desc[ostart + ori1] += cw1; desc[ostart + ori2] += cw2;
        }
    }
}

/* describeURWithoutNormalization / describeApproxWithoutNormalization
 * (surfd.cu:1566-1615, 2391-2444 with addUprightSample 1288-1317 and
 * addSample 1984-2015), then normalize (surfd.cu:2447-2493). */
void or_describe(const or_param* p, const or_geom* g, const int32_t* ii,
                 const float lut2[40], const or_point* pt, float* desc)
{
    const int nf = p->nfeatures, wsz = p->desc_wsz, osz = p->orient_size;
    const int ip = g->iwhp.z;
    memset(desc, 0, sizeof(float) * nf);
    /* doubled: (2x, 2y) and 3.3 * scale in the doubled integral image
     * (surfd.cu:1581-1592 upright, 2406-2417 rotated) */
    const float x = p->doubled ? pt->x + pt->x : pt->x;
    const float y = p->doubled ? pt->y + pt->y : pt->y;
    const float scale = p->doubled ? 3.3f * pt->scale : 1.65f * pt->scale;
    const int step = f2i_rn(scale * 0.5f) > 1 ? f2i_rn(scale * 0.5f) : 1;
    const int ix = f2i_rn(x), iy = f2i_rn(y);
    const float spacing = scale * (float)p->mag_factor;
    const int hs = f2i_rz(scale);
    const float wofs = (float)wsz * 0.5f - 0.5f;
    const float fw = (float)wsz;
    if (p->upright) {
        const float dx0 = x - (float)ix;
        const float dy0 = y - (float)iy;
        const int iradius = f2i_rn(((spacing * (float)(wsz + 1)) * 0.5f) / (float)step);
        for (int i = -iradius; i <= iradius; i++) {
            for (int j = -iradius; j <= iradius; j++) {
                const float rpos = ((float)(step * i) - dy0) / spacing;
                const float cpos = ((float)(step * j) - dx0) / spacing;
                const float rx = rpos + wofs, cx = cpos + wofs;
                if (!(rx > -1.f && rx < fw && cx > -1.f && cx < fw)) continue;
                const int r = iy + i * step, c = ix + j * step;
                if (!(r >= 1 + hs && r < g->iwhp.y - 1 - hs && c >= 1 + hs && c < g->iwhp.x - 1 - hs)) continue;
                const float rr = rpos * rpos, cc = cpos * cpos;
                const float weight = lut2[f2i_rz(rr + cc)];
                const float dx = (weight * (float)wavelet2(ii, c, r, hs, ip)) * INV255;
                const float dy = (weight * (float)wavelet1(ii, c, r, hs, ip)) * INV255;
                if (!p->extend) {
                    place(desc, wsz, osz, dx, (dx < 0 ? 0 : 1), dy, (dy < 0 ? 2 : 3), rx, cx);
                } else {
                    place(desc, wsz, osz, dx, (dy < 0 ? 0 : 1), fabsf(dx), (dy < 0 ? 2 : 3), rx, cx);
                    place(desc, wsz, osz, dy, (dx < 0 ? 4 : 5), fabsf(dy), (dx < 0 ? 6 : 7), rx, cx);
                }
            }
        }
    } else {
        const float fracx = x - (float)ix;
        const float fracy = y - (float)iy;
        const float sine = or_sinf(pt->ori);
        const float cose = or_cosf(pt->ori);
        const float fracc = ((-sine) * fracy) + (cose * fracx);
        const float fracr = (cose * fracy) + (sine * fracx);
        const int iradius = f2i_rn((((1.4f * spacing) * (float)(wsz + 1)) * 0.5f) / (float)step);
        const float fstep = (float)step;
        for (int i = -iradius; i <= iradius; i++) {
            for (int j = -iradius; j <= iradius; j++) {
                const float fi = (float)i, fj = (float)j;
                const float a1 = cose * fi, b1 = sine * fj;
                const float a2 = (-sine) * fi, b2 = cose * fj;
                const float rpos = ((fstep * (a1 + b1)) - fracr) / spacing;
                const float cpos = ((fstep * (a2 + b2)) - fracc) / spacing;
                const float rx = rpos + wofs, cx = cpos + wofs;
                if (!(rx > -1.f && rx < fw && cx > -1.f && cx < fw)) continue;
                const int r = iy + i * step, c = ix + j * step;
                if (!(r >= 1 + hs && r < g->iwhp.y - 1 - hs && c >= 1 + hs && c < g->iwhp.x - 1 - hs)) continue;
                const float rr = rpos * rpos, cc = cpos * cpos;
                const float weight = lut2[f2i_rz(rr + cc)];
                const float dxx = (weight * (float)wavelet2(ii, c, r, hs, ip)) * INV255;
                const float dyy = (weight * (float)wavelet1(ii, c, r, hs, ip)) * INV255;
                const float dx = (cose * dxx) + (sine * dyy);
                const float dy = (sine * dxx) - (cose * dyy);
                if (!p->extend) {
                    place(desc, wsz, osz, dx, (dx < 0 ? 0 : 1), dy, (dy < 0 ? 2 : 3), rx, cx);
                } else {
                    place(desc, wsz, osz, dx, (dy < 0 ? 0 : 1), fabsf(dx), (dy < 0 ? 2 : 3), rx, cx);
                    place(desc, wsz, osz, dy, (dx < 0 ? 4 : 5), fabsf(dy), (dx < 0 ? 6 : 7), rx, cx);
                }
            }
        }
    }
    /* normalize (surfd.cu:2447-2493): the squares, zero-padded to
     * P = max(64, next power of two >= nf), summed by the sequential-
     * addressing tree (strides P/2 .. 1).  For nf = 64 / 128 -- the sizes of
     * desc_wsz 4 -- this is the reference's order exactly (its stride loop
     * down to 64, then the warp-synchronous 32 .. 1).  For other window
     * sizes the reference reads its nfeatures-float shared array out of
     * bounds (tid + 32 >= nf) or, when nf is not a power of two (72, 100,
     * 200, ...), adds some squares twice; here it is defined as the full sum,
     * which the HIP kernels compute too. */
    float sq[512];
    int P = 64;
    while (P < nf) P <<= 1;
    for (int t = 0; t < P; t++) sq[t] = t < nf ? desc[t] * desc[t] : 0.f;
    for (int stride = P / 2; stride >= 1; stride >>= 1)
        for (int t = 0; t < stride; t++) sq[t] = sq[t] + sq[t + stride];
    const float fac = 1.f / sqrtf(sq[0]);
    for (int t = 0; t < nf; t++) desc[t] = desc[t] * fac;
}

/* ---------------------------------------------------------- full frame */

int or_detect_and_compute(const or_param* p, const uint8_t* img, int w, int h,
                          int pitch, or_point* pts, int max_pts, float* desc,
                          int* n_candidates)
{
    or_geom g;
    or_octave oct[OR_MAX_OCTAVE];
    or_geometry(p, w, h, &g);
    or_octave_params(p, &g, oct);
    int32_t* ii = (int32_t*)calloc((size_t)g.iwhp.y * g.iwhp.z, sizeof(int32_t));
    float* resp = (float*)calloc(g.tot_osize, sizeof(float));
    if (!ii || !resp) { free(ii); free(resp); return -1; }
    if (p->doubled) {                                 /* surf.cpp:234-235 */
        if (w < 2 || h < 2) { free(ii); free(resp); return -1; }
        const int dp = g.iwhp.z;
        uint8_t* dimg = (uint8_t*)malloc((size_t)(2 * h - 2) * dp);
        if (!dimg) { free(ii); free(resp); return -1; }
        or_double_image(img, w, h, pitch, dimg, dp);
        or_integral(dimg, 2 * w - 2, 2 * h - 2, dp, ii, g.iwhp.z);
        free(dimg);
    } else {
        or_integral(img, w, h, pitch, ii, g.iwhp.z);
    }
    or_hessian(p, &g, oct, ii, resp);
    int cand = or_find_points(p, &g, oct, ii, resp, pts, max_pts);
    int n = cand < max_pts ? cand : max_pts;
    if (n_candidates) *n_candidates = cand;
    if (desc) {
        float lut1[83], lut2[40], bins[OR_NBIN];
        or_init_tables(lut1, lut2, bins);
        for (int i = 0; i < n; i++) {
            if (!p->upright) pts[i].ori = or_orientation(p, &g, ii, lut1, bins, &pts[i]);
            or_describe(p, &g, ii, lut2, &pts[i], desc + (size_t)i * p->nfeatures);
        }
    }
    free(ii);
    free(resp);
    return n;
}

/* ---------------------------------------------------------- CPU baseline */

typedef struct {
    const or_param* p;
    const uint8_t* frames;
    int w, h, pitch, max_pts, nframes, nthreads, tid;
    size_t stride;
    long long pts;
} or_job;

static void* or_worker(void* arg)
{
    or_job* j = (or_job*)arg;
    or_point* pts = (or_point*)malloc(sizeof(or_point) * (size_t)j->max_pts);
    float* desc = (float*)malloc(sizeof(float) * (size_t)j->max_pts * j->p->nfeatures);
    for (int f = j->tid; f < j->nframes; f += j->nthreads) {
        int n = or_detect_and_compute(j->p, j->frames + (size_t)f * j->stride, j->w, j->h,
                                      j->pitch, pts, j->max_pts, desc, NULL);
        if (n > 0) j->pts += n;
    }
    free(pts);
    free(desc);
    return NULL;
}

double or_bench_frames(const or_param* p, const uint8_t* frames, int nframes,
                       int w, int h, int pitch, size_t frame_stride,
                       int max_pts, int nthreads, long long* total_pts)
{
    if (nthreads < 1) nthreads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    or_job* jobs = (or_job*)calloc(nthreads, sizeof(or_job));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (or_job){p, frames, w, h, pitch, max_pts, nframes, nthreads, t, frame_stride, 0};
        pthread_create(&th[t], NULL, or_worker, &jobs[t]);
    }
    long long tot = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        tot += jobs[t].pts;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(th);
    free(jobs);
    if (total_pts) *total_pts = tot;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ------------------------------------------------------- KAT hooks */
void or_test_solve3(float sol[3], float sq[9])
{
    float m[3][3];
    for (int i = 0; i < 9; i++) m[i / 3][i % 3] = sq[i];
    solve3(sol, m);
    for (int i = 0; i < 9; i++) sq[i] = m[i / 3][i % 3];
}
float or_test_fit(const float* src, float off[3], int s, int r, int c, int osize, int sp)
{
    return fit_quadratic(src, off, s, r, c, osize, sp);
}
uint32_t or_test_box(const int32_t* ii, int ipitch, int x1, int y1, int x2, int y2)
{
    return box(ii, x1, y1, x2, y2, ipitch);
}
void or_test_place(float* desc, int wsz, int osz, float mag1, int ori1, float mag2, int ori2, float rx, float cx)
{
    place(desc, wsz, osz, mag1, ori1, mag2, ori2, rx, cx);
}

/* ------------------------------------------------------------- match --
 * Surfor::match -> cuFindMaxCorr -> findMaxCorr (surf.cpp:418-428,
 * surfd.cu:3554-3566, 2530-2656), restated per point of set 1.
 *
 * The reference block holds 32 points of set 1; its 8 thread rows (ty) each
 * scan the set-2 points p2 with (p2 % 32) / 4 == ty of every FULL 32-point
 * tile (`bp2 < num_pts2 - M7H + 1`, surfd.cu:2569: the last partial tile is
 * dropped), in increasing p2, keeping (max, second, index) with strict `>`
 * from (0, 0, -1) (surfd.cu:2607-2621).  Every score is one sequential fp32
 * FMA chain over the descriptor (nvcc contracts `score += a * b`,
 * surfd.cu:2596-2601, CMakeLists.txt passes no --fmad=false).  Row 0's
 * state is then merged with rows 1..7 in order, ignoring the rows' second
 * scores and rows whose index equals the running one (surfd.cu:2638-2655).
 * Defined where the reference is not: points p1 >= n1 are not written
 * (the reference writes a whole 32-point block), and index -1 (no positive
 * score) gives match_x = match_y = 0 instead of reading surf2[-1].
 * full_tail != 0 also scans the last partial tile (fixes the tile-tail bug;
 * an option, the default follows the reference). */
void or_match(or_point* pts1, const or_point* pts2, const float* f1, const float* f2,
              int n1, int n2, int nf, int full_tail)
{
    const int ntile = full_tail ? (n2 + 31) / 32 : n2 / 32;
    for (int p1 = 0; p1 < n1; p1++) {
        const float* a = f1 + (size_t)p1 * nf;
        float gmax[8], gsec[8];
        int gidx[8];
        for (int g = 0; g < 8; g++) {
            float mx = 0.0f, sc = 0.0f;
            int ix = -1;
            for (int t = 0; t < ntile; t++) {
                for (int dy = 0; dy < 4; dy++) {
                    const int p2 = 32 * t + 4 * g + dy;
                    if (p2 >= n2) continue;
                    const float* b = f2 + (size_t)p2 * nf;
                    float s = 0.0f;
                    for (int d = 0; d < nf; d++) s = fmaf(a[d], b[d], s);
                    if (s > mx) { sc = mx; mx = s; ix = p2; }
                    else if (s > sc) sc = s;
                }
            }
            gmax[g] = mx; gsec[g] = sc; gidx[g] = ix;
        }
        float mx = gmax[0], sc = gsec[0];
        int ix = gidx[0];
        for (int g = 1; g < 8; g++) {
            if (ix == gidx[g]) continue;
            if (gmax[g] > mx) { sc = fmaxf(mx, sc); mx = gmax[g]; ix = gidx[g]; }
            else if (gmax[g] > sc) sc = gmax[g];
        }
        or_point* q = &pts1[p1];
        q->score = mx;
        q->match = ix;
        q->match_x = ix >= 0 ? pts2[ix].x : 0.0f;
        q->match_y = ix >= 0 ? pts2[ix].y : 0.0f;
        q->ambiguity = sc / (mx + 1e-6f);
    }
}

/* Checker for the HIP kernels' descriptor-position quotient (div_by in
 * surfhip_kernels.hip: q0 = x r, q = fma(fma(-q0, y, x), r, q0) with r =
 * 1 / y): counts, over n pseudo-random (x, y) in the ranges the descriptor
 * kernels see (y = 3 * (1.65 * scale), scale in [1, 80); |x| < 400, or any
 * normal |x| >= 2^-100 against y of every exponent 2^1 .. 2^8 with random or
 * all-ones significands), the trials where q differs from the IEEE x / y.
 * Test infrastructure only. */
long or_div_by_mismatches(long n, uint64_t seed)
{
    uint64_t s = seed | 1u;
    long bad = 0;
    for (long i = 0; i < n; i++) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const uint64_t a = s;
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const uint64_t b = s;
        float x, y;
        if (i & 1) {
            const float scale = 1.f + (float)(a % 1000000u) * 7.9e-5f;
            y = 3.0f * (1.65f * scale);
            x = ((float)((int64_t)(b % 8000001u) - 4000000)) * 1e-4f;
        } else {
            const uint32_t m = (a & 1u) ? 0x7FFFFFu - (uint32_t)((a >> 1) % 2048u) : (uint32_t)((a >> 1) & 0x7FFFFFu);
            const uint32_t e = 128u + (uint32_t)((a >> 40) % 8u);
            const uint32_t yu = (e << 23) | m;
            const uint32_t xu = (0x0D800000u + (uint32_t)(b % (0x43800000u - 0x0D800000u))) | ((uint32_t)(b >> 63) << 31);
            memcpy(&y, &yu, 4);
            memcpy(&x, &xu, 4);
        }
        volatile float yy = y;
        const float r = 1.0f / yy;
        const float q0 = x * r;
        const float q = fmaf(fmaf(-q0, y, x), r, q0);
        const float ref = x / yy;
        if (q != ref) bad++;
    }
    return bad;
}
