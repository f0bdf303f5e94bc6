// surfhip_match.hip -- descriptor matching (Surfor::match) for gfx950.
//
// Reference: Surfor::match (surf.cpp:418-428) -> cuFindMaxCorr
// (surfd.cu:3554-3566) -> findMaxCorr (surfd.cu:2530-2656).  For every
// point p1 of set 1 the reference keeps, per thread row ty = 0..7 of its
// block, the (max, second, index) of the scores against the set-2 points p2
// with (p2 % 32) / 4 == ty of every FULL 32-point tile (surfd.cu:2569 drops
// the last partial tile), then merges row 0 with rows 1..7 in order
// (surfd.cu:2638-2655).  A score is one fp32 FMA chain over the descriptor
// in index order (nvcc contracts `score += a * b`, surfd.cu:2596-2601).
//
// The same result, laid out for CDNA4 instead of a 32x8 CUDA block:
//   * k_match_part: lane = p1 (its descriptor lives in VGPRs), the wave walks
//     a chunk of set-2 tiles with the p2 descriptor wave-uniform (scalar
//     loads, an SGPR operand of every v_fma_f32), one FMA chain per score,
//     the 8 row states (max, second, index) in registers -- the tile position
//     j of an unrolled 32-step loop fixes the row, j / 4.  grid.y splits set
//     2 into chunks so that a few thousand points fill the 256 CUs.
//   * k_match_merge: one thread per (p1, row): the chunk states of the row
//     are combined in chunk order (top-2 of a concatenation, earlier index on
//     a tie: exactly the sequential scan's result); the row-0 lane then does
//     the reference's row merge over lane shuffles and writes the five
//     SurfPoint fields.
// No dense-contraction unit is used: MFMA would re-associate the sums and
// break bit-exact scores (and so argmax ties); at ~3k x 3k x 64 the FMA
// chains cost tens of microseconds.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "surfhip_internal.h"

namespace surfhip {

namespace {

constexpr int kMatchThreads = 256;
constexpr int kTilesPerChunk = 2;   // 64 set-2 points per chunk (2 waves / SIMD at 3k x 3k)

// Sequential (max, second, index) update with strict '>' (surfd.cu:2611-2620),
// branch-free (selects, no divergent control flow around the state).
__device__ __forceinline__ void scan_update(float s, int p2, float& mx, float& sc, int& ix)
{
    const bool gt = s > mx;
    const bool gt2 = s > sc;
    sc = gt ? mx : (gt2 ? s : sc);
    mx = gt ? s : mx;
    ix = gt ? p2 : ix;
}

template <int NF>
__global__ __launch_bounds__(kMatchThreads) void k_match_part(const float* __restrict__ f1,
                                                              const float* __restrict__ f2, int n1, int nscan,
                                                              int ntile, float* __restrict__ pmx,
                                                              float* __restrict__ psc, int* __restrict__ pix)
{
    const int p1 = blockIdx.x * kMatchThreads + threadIdx.x;
    const int q1 = p1 < n1 ? p1 : n1 - 1;
    float a[NF];
    const float4* ap = reinterpret_cast<const float4*>(f1 + (size_t)q1 * NF);
#pragma unroll
    for (int d = 0; d < NF / 4; ++d) {
        const float4 v = ap[d];
        a[4 * d] = v.x;
        a[4 * d + 1] = v.y;
        a[4 * d + 2] = v.z;
        a[4 * d + 3] = v.w;
    }
    float mx[8], sc[8];
    int ix[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        mx[g] = 0.0f;
        sc[g] = 0.0f;
        ix[g] = -1;
    }
    const int t0 = blockIdx.y * kTilesPerChunk;
    const int t1 = min(t0 + kTilesPerChunk, ntile);
    for (int t = t0; t < t1; ++t) {
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const int p2 = 32 * t + j;
            if (p2 < nscan) {
                const float* b = f2 + (size_t)p2 * NF;
                float s = 0.0f;
#pragma unroll
                for (int d = 0; d < NF; ++d) s = __builtin_fmaf(a[d], b[d], s);
                scan_update(s, p2, mx[j >> 2], sc[j >> 2], ix[j >> 2]);
            }
        }
    }
    if (p1 < n1) {
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            const size_t o = ((size_t)blockIdx.y * n1 + p1) * 8 + g;
            pmx[o] = mx[g];
            psc[o] = sc[g];
            pix[o] = ix[g];
        }
    }
}

// Any descriptor length (a multiple of 4, <= 1024): runtime trip count.
__global__ __launch_bounds__(kMatchThreads) void k_match_part_any(const float* __restrict__ f1,
                                                                  const float* __restrict__ f2, int n1, int nf,
                                                                  int nscan, int ntile, float* __restrict__ pmx,
                                                                  float* __restrict__ psc, int* __restrict__ pix)
{
    const int p1 = blockIdx.x * kMatchThreads + threadIdx.x;
    const int q1 = p1 < n1 ? p1 : n1 - 1;
    const float* a = f1 + (size_t)q1 * nf;
    float mx[8], sc[8];
    int ix[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        mx[g] = 0.0f;
        sc[g] = 0.0f;
        ix[g] = -1;
    }
    const int t0 = blockIdx.y * kTilesPerChunk;
    const int t1 = min(t0 + kTilesPerChunk, ntile);
    for (int t = t0; t < t1; ++t) {
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const int p2 = 32 * t + j;
            if (p2 < nscan) {
                const float* b = f2 + (size_t)p2 * nf;
                float s = 0.0f;
                for (int d = 0; d < nf; ++d) s = __builtin_fmaf(a[d], b[d], s);
                scan_update(s, p2, mx[j >> 2], sc[j >> 2], ix[j >> 2]);
            }
        }
    }
    if (p1 < n1) {
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            const size_t o = ((size_t)blockIdx.y * n1 + p1) * 8 + g;
            pmx[o] = mx[g];
            psc[o] = sc[g];
            pix[o] = ix[g];
        }
    }
}

// One thread per (p1, row g): lanes 8 q .. 8 q + 7 of a wave hold the 8 rows
// of one p1; the row-0 lane then merges the others in row order.
__global__ __launch_bounds__(256) void k_match_merge(surfhip_point* __restrict__ pts1,
                                                     const surfhip_point* __restrict__ pts2, int n1, int nchunk,
                                                     const float* __restrict__ pmx, const float* __restrict__ psc,
                                                     const int* __restrict__ pix)
{
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int p1 = tid >> 3, g = tid & 7;
    const bool live = p1 < n1;
    // Row g over all chunks, in chunk (= p2) order: top-2 of the
    // concatenated sequences, the earlier index kept on a tie.
    float mx = 0.0f, sc = 0.0f;
    int ix = -1;
    if (live) {
#pragma unroll 8
        for (int c = 0; c < nchunk; ++c) {
            const size_t o = ((size_t)c * n1 + p1) * 8 + g;
            const float bm = pmx[o], bs = psc[o];
            const int bi = pix[o];
            const bool gt = bm > mx;
            sc = gt ? fmaxf(mx, bs) : fmaxf(sc, bm);
            mx = gt ? bm : mx;
            ix = gt ? bi : ix;
        }
    }
    // Row merge (surfd.cu:2638-2655): row 0 starts the state, the rows'
    // second scores are not used, equal indices are skipped.
    float M = mx, S = sc;
    int I = ix;
#pragma unroll
    for (int r = 1; r < 8; ++r) {
        const float rm = __shfl(mx, (threadIdx.x & ~7) + r);
        const int ri = __shfl(ix, (threadIdx.x & ~7) + r);
        if (I != ri) {
            if (rm > M) {
                S = fmaxf(M, S);
                M = rm;
                I = ri;
            } else if (rm > S) {
                S = rm;
            }
        }
    }
    if (!live || g != 0) return;
    surfhip_point& q = pts1[p1];
    q.score = M;
    q.match = I;
    q.match_x = I >= 0 ? pts2[I].x : 0.0f;
    q.match_y = I >= 0 ? pts2[I].y : 0.0f;
    q.ambiguity = S / (M + 1e-6f);
}

}  // namespace

size_t match_scratch_bytes(int n1, int n2, int flags)
{
    const int nscan = (flags & SURFHIP_MATCH_FULL_TAIL) ? n2 : 32 * (n2 / 32);
    const int ntile = (nscan + 31) / 32;
    const int nchunk = ntile > 0 ? (ntile + kTilesPerChunk - 1) / kTilesPerChunk : 0;
    return (size_t)nchunk * 8 * (size_t)n1 * 12;
}

hipError_t launch_match(surfhip_point* pts1, const surfhip_point* pts2, const float* f1, const float* f2, int n1,
                        int n2, int nf, int flags, void* scratch, hipStream_t s)
{
    const int nscan = (flags & SURFHIP_MATCH_FULL_TAIL) ? n2 : 32 * (n2 / 32);
    const int ntile = (nscan + 31) / 32;
    const int nchunk = ntile > 0 ? (ntile + kTilesPerChunk - 1) / kTilesPerChunk : 0;
    float* pmx = static_cast<float*>(scratch);
    float* psc = pmx + (size_t)nchunk * 8 * n1;
    int* pix = reinterpret_cast<int*>(psc + (size_t)nchunk * 8 * n1);
    if (nchunk > 0) {
        const dim3 grid((n1 + kMatchThreads - 1) / kMatchThreads, nchunk);
        if (nf == 64)
            k_match_part<64><<<grid, kMatchThreads, 0, s>>>(f1, f2, n1, nscan, ntile, pmx, psc, pix);
        else if (nf == 128)
            k_match_part<128><<<grid, kMatchThreads, 0, s>>>(f1, f2, n1, nscan, ntile, pmx, psc, pix);
        else
            k_match_part_any<<<grid, kMatchThreads, 0, s>>>(f1, f2, n1, nf, nscan, ntile, pmx, psc, pix);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    k_match_merge<<<(8 * n1 + 255) / 256, 256, 0, s>>>(pts1, pts2, n1, nchunk, pmx, psc, pix);
    return hipGetLastError();
}

}  // namespace surfhip
