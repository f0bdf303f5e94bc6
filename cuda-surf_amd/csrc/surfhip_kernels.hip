// surfhip_kernels.hip -- gfx950 kernels of the SURF detect+describe path.
//
// Stage map (reference file:line -> kernel here):
//   integralRow/integralCol   surfd.cu:129-165, 2683-2704  -> k_ii_bandsum, k_ii_bandscan, k_ii_fill
//   halfImage                 surfd.cu:321-331             -> virtual planes read by k_nms (OctView)
//   calcHessianMultiConst     surfd.cu:445-481, 2829-2894  -> k_hessian
//   findMaximumWithInterp     surfd.cu:676-832, 3058-3079  -> k_nms
//   (atomicInc emission order) surfd.cu:825-830            -> k_sort (canonical order + max_pts cap)
//   assignOrientationApprox   surfd.cu:1711-1960           -> k_describe<rotated>, phase 1
//   describe*WithoutNormalization + normalize
//                             surfd.cu:1566-1615, 2391-2493 -> k_describe, phases 2-3
//
// Numerics: this file is compiled with -ffp-contract=off and the pragma
// below, so each written float operation rounds once (the oracle's
// semantics); explicit fmaf() only where the reference wrote __fmaf_rn.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <type_traits>
#include <utility>

#include "surfhip_internal.h"

namespace surfhip {

#define INV255 0.003921568627f          // surfd.cu:356
#define H_PI_F 1.5707963267948966f      // cuda_utils.h:8
#define SEP_ANGLE_F 0.08726646259971647f
#define WINDOW_F 1.0471975511965976f
#define M_PI_D 3.14159265358979323846

__constant__ Tables c_tab;

hipError_t set_tables(const Tables& t)
{
    return hipMemcpyToSymbol(HIP_SYMBOL(c_tab), &t, sizeof(Tables), 0, hipMemcpyHostToDevice);
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) is per device: remember
// per (kernel, device) that it was set (a process may drive several GPUs,
// from several threads)
hipError_t set_max_lds(const void* fn, int bytes)
{
    constexpr int kFns = 8, kDevs = 64;
    static const void* fns[kFns] = {};
    static std::atomic<unsigned long long> done[kFns];
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kDevs) return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    static std::mutex mu;
    int slot = -1;
    {
        std::lock_guard<std::mutex> lk(mu);
        for (int i = 0; i < kFns && slot < 0; i++)
            if (fns[i] == fn || fns[i] == nullptr) {
                fns[i] = fn;
                slot = i;
            }
    }
    if (slot < 0) return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    const unsigned long long bit = 1ull << dev;
    if (done[slot].load(std::memory_order_acquire) & bit) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done[slot].fetch_or(bit, std::memory_order_release);
    return e;
}

__device__ __forceinline__ int f2i_rn(float v) { return (int)__builtin_rintf(v); }
__device__ __forceinline__ int f2i_rz(float v) { return (int)v; }

// Where a keypoint is described: a doubled detector's integral image is of
// the 2x frame, so the reference samples it at (2x, 2y) with 3.3 * scale
// for the descriptor (surfd.cu:1581-1592, 2406-2417) and 2 * scale for the
// orientation (surfd.cu:1734-1745); otherwise (x, y) and 1.65 * scale.
struct DescAt {
    float x, y, scale;
};
template <typename PT>
__device__ __forceinline__ DescAt desc_at(int doubled, const PT& p)
{
    return doubled ? DescAt{p.x + p.x, p.y + p.y, 3.3f * p.scale} : DescAt{p.x, p.y, 1.65f * p.scale};
}
template <typename PT>
__device__ __forceinline__ DescAt ori_at(int doubled, const PT& p)
{
    return doubled ? DescAt{p.x + p.x, p.y + p.y, p.scale + p.scale} : DescAt{p.x, p.y, p.scale};
}

__device__ __forceinline__ unsigned lane_id()
{
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// Buffer (SRD) memory ops.  A raw buffer load past num_records returns 0 and
// a store past it is dropped, so loads and stores at image edges need no
// branch: a branch around a load makes hipcc wait for it (vmcnt(0)) right
// there, which serialises a prefetch pipeline, and a store under a divergent
// branch makes the outstanding-op count unknown, so the next counted wait
// becomes vmcnt(0) too.  Descriptors are built from wave-uniform values only.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));
typedef float v2f32 __attribute__((ext_vector_type(2)));
// 3 x mod 2^32 as one full-rate v_lshl_add_u32: LLVM lowers `3u * x` to
// the quarter-rate v_mul_lo_u32 / v_mad_u64_u32, which made up about a
// quarter of the Hessian kernels' VALU issue time
__device__ __forceinline__ uint32_t mul3(uint32_t x)
{
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 1, %1" : "=v"(r) : "v"(x));
    return r;
}
constexpr uint32_t kOOB = 0x80000000u;          // byte offset past every buffer here

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, long long bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 buf_ld4(rsrc_t r, uint32_t off)
{
    const v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return make_uint4(v.x, v.y, v.z, v.w);
}
// streaming store (nt): response planes are read back only by the NMS pass
__device__ __forceinline__ void buf_st_nt(rsrc_t r, uint32_t off, float v)
{
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 2);
}

// compile-time loop: fn(std::integral_constant<int, K>) for K = 0 .. N-1
template <typename Fn, int... Ks>
__device__ __forceinline__ void static_for_seq(Fn&& fn, std::integer_sequence<int, Ks...>)
{
    (fn(std::integral_constant<int, Ks>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void static_for(Fn&& fn)
{
    static_for_seq(fn, std::make_integer_sequence<int, N>{});
}

// LDS ordering between the lanes of one wave, no wait: the LDS executes one
// wave's DS instructions in issue order, so a ds_read issued after a
// ds_write of the same wave sees it (and a later write cannot overtake an
// earlier read); only the compiler must keep the order.
__device__ __forceinline__ void lds_order()
{
    asm volatile("" ::: "memory");
}

// LDS visibility between the lanes of one wave
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ======================================================================
// Integral image.  Three passes over row bands of kBandRows rows:
//  (A) k_ii_bandsum : per band, per column, the sum of the band's pixels
//  (B) k_ii_bandscan: exclusive prefix over bands -> column sums above band
//  (C) k_ii_fill    : the band's first integral row is the exclusive row
//      scan of (B); each further row adds the exclusive row scan of the
//      pixels.  u8 is read twice, the int32 image written once.
// Semantics of integralRow/integralCol (surfd.cu:129-165): ii[y+1][x+1] is
// the sum over rows <= y, cols <= x; row 0 / col 0 are 0 (written here).
// uint32 arithmetic wraps exactly like the reference's int adds.
// ======================================================================

template <int CPT>
__device__ __forceinline__ void load_px(const uint8_t* row, int x0, int W, uint32_t (&px)[CPT])
{
    if constexpr (CPT == 8) {
        const uint2 v = *reinterpret_cast<const uint2*>(row + x0);
        const uint32_t w[2] = {v.x, v.y};
#pragma unroll
        for (int k = 0; k < 8; k++) px[k] = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
    } else if constexpr (CPT == 32) {
        const uint4 a = *reinterpret_cast<const uint4*>(row + x0);
        // the second half only where it holds frame columns: the caller's
        // pitch is a multiple of 16, not of 32, so x0 + 16 >= W may lie past
        // the row (and past the buffer on the last row)
        const uint4 b = (x0 + 16 < W) ? *reinterpret_cast<const uint4*>(row + x0 + 16) : make_uint4(0u, 0u, 0u, 0u);
        const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int k = 0; k < 32; k++) px[k] = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
    } else {
        const uint4 v = *reinterpret_cast<const uint4*>(row + x0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 16; k++) px[k] = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
    }
#pragma unroll
    for (int k = 0; k < CPT; k++)
        if (x0 + k >= W) px[k] = 0u;
}

template <int CPT>
__global__ __launch_bounds__(256) void k_ii_bandsum(const uint8_t* __restrict__ frames, int pitch,
                                                    long long fstride, int W, int H, int nbands,
                                                    uint32_t* __restrict__ colsum, int CW, int br)
{
    const int band = blockIdx.x, f = blockIdx.y;
    const int x0 = threadIdx.x * CPT;
    if (x0 >= W) return;
    const int y0 = band * br;
    const int rows = min(br, H - y0);
    const uint8_t* src = frames + (size_t)f * fstride + (size_t)y0 * pitch;
    uint32_t acc[CPT];
#pragma unroll
    for (int k = 0; k < CPT; k++) acc[k] = 0u;
    // 8 rows' loads in flight per iteration (rows past the band re-read the
    // band's last row and are not added)
    for (int r0 = 0; r0 < rows; r0 += 8) {
        uint32_t px[8][CPT];
#pragma unroll
        for (int d = 0; d < 8; d++) load_px<CPT>(src + (size_t)min(r0 + d, rows - 1) * pitch, x0, W, px[d]);
#pragma unroll
        for (int d = 0; d < 8; d++)
            if (r0 + d < rows) {
#pragma unroll
                for (int k = 0; k < CPT; k++) acc[k] += px[d][k];
            }
    }
    uint32_t* dst = colsum + ((size_t)f * nbands + band) * CW + x0;
#pragma unroll
    for (int k = 0; k < CPT; k += 4)
        *reinterpret_cast<uint4*>(dst + k) = make_uint4(acc[k], acc[k + 1], acc[k + 2], acc[k + 3]);
}

template <int CH>
__global__ __launch_bounds__(256) void k_ii_bandscan(uint32_t* __restrict__ colsum, int nbands, int CW, int W)
{
    const int x = blockIdx.x * 256 + threadIdx.x, f = blockIdx.y;
    if (x >= W) return;
    uint32_t* c = colsum + (size_t)f * nbands * CW + x;
    uint32_t run = 0u;
    // CH bands' loads in flight per chunk (one memory latency per chunk, not
    // per band): 48 for the 32-row bands of a batch, 136 for the 8-row bands
    // of a single 1080p frame (135 bands: 9 round trips at 16, 12 us,
    // profiles/r05ac2_kernel_stats.csv)
    for (int b0 = 0; b0 < nbands; b0 += CH) {
        uint32_t v[CH];
#pragma unroll
        for (int k = 0; k < CH; k++) v[k] = (b0 + k < nbands) ? c[(size_t)(b0 + k) * CW] : 0u;
#pragma unroll
        for (int k = 0; k < CH; k++)
            if (b0 + k < nbands) {
                c[(size_t)(b0 + k) * CW] = run;
                run += v[k];
            }
    }
}

// Exclusive scan across the 256-thread block of CPT consecutive values per
// thread (wave64 shuffle scan + LDS exchange of the 4 wave totals).
template <int CPT>
__device__ __forceinline__ void block_excl_scan(uint32_t (&v)[CPT], uint32_t* lds4)
{
    uint32_t run = 0u;
#pragma unroll
    for (int k = 0; k < CPT; k++) {
        const uint32_t t = v[k];
        v[k] = run;
        run += t;
    }
    const unsigned lane = lane_id();
    const int wave = threadIdx.x >> 6;
    uint32_t inc = run;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t n = (uint32_t)__shfl_up((int)inc, d, 64);
        if (lane >= (unsigned)d) inc += n;
    }
    if (lane == 63) lds4[wave] = inc;
    __syncthreads();
    uint32_t base = inc - run;
    for (int w = 0; w < wave; w++) base += lds4[w];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CPT; k++) v[k] += base;
}

template <int CPT>
__global__ __launch_bounds__(256) void k_ii_fill(const uint8_t* __restrict__ frames, int pitch,
                                                 long long fstride, int W, int H, int nbands,
                                                 const uint32_t* __restrict__ colpre, int CW,
                                                 int32_t* __restrict__ ii, int ip, long long istride, int br)
{
    __shared__ uint32_t lds4[4];
    const int band = blockIdx.x, f = blockIdx.y;
    const int x0 = threadIdx.x * CPT;
    const bool active = x0 <= W;               // thread owns integral columns x0..x0+CPT-1
    const int y0 = band * br;
    const int rows = min(br, H - y0);
    uint32_t acc[CPT];
    {
        const uint32_t* c = colpre + ((size_t)f * nbands + band) * CW;
#pragma unroll
        for (int k = 0; k < CPT; k++) acc[k] = (x0 + k < W) ? c[x0 + k] : 0u;
    }
    block_excl_scan<CPT>(acc, lds4);           // acc = ii[y0][x0 + k]
    uint32_t* out = reinterpret_cast<uint32_t*>(ii) + (size_t)f * istride;
    if (band == 0 && active) {
#pragma unroll
        for (int k = 0; k < CPT; k += 4)
            *reinterpret_cast<uint4*>(out + x0 + k) = make_uint4(0u, 0u, 0u, 0u);
    }
    const uint8_t* src = frames + (size_t)f * fstride + (size_t)y0 * pitch;
    for (int r = 0; r < rows; r++) {
        uint32_t px[CPT];
        if (x0 < W) load_px<CPT>(src + (size_t)r * pitch, x0, W, px);
        else {
#pragma unroll
            for (int k = 0; k < CPT; k++) px[k] = 0u;
        }
        block_excl_scan<CPT>(px, lds4);
#pragma unroll
        for (int k = 0; k < CPT; k++) acc[k] += px[k];
        if (active) {
            // pad columns (> W) stay zero: the flat reads of getTrace can
            // land on them (see trace_sign)
            uint32_t o[CPT];
#pragma unroll
            for (int k = 0; k < CPT; k++) o[k] = (x0 + k <= W) ? acc[k] : 0u;
            uint32_t* dst = out + (size_t)(y0 + r + 1) * ip + x0;
#pragma unroll
            for (int k = 0; k < CPT; k += 4)
                *reinterpret_cast<uint4*>(dst + k) = make_uint4(o[k], o[k + 1], o[k + 2], o[k + 3]);
        }
    }
}

// Pass (C) with one wave per band and no barriers: lane l owns columns
// 4 l + 256 t + j (t < NT, j < 4), so every load is 256 contiguous bytes and
// every store 1 KiB; the row scan is NT wave scans with a running carry.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp_add(uint32_t v)
{
    return v + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWMASK, 0xf, false);
}
// inclusive scan over the wave's 64 lanes (gfx9 DPP: row shifts, then the
// row_bcast:15 / row_bcast:31 carries) -- six VALU ops, no LDS round trip
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
    v = dpp_add<0x111, 0xf>(v);
    v = dpp_add<0x112, 0xf>(v);
    v = dpp_add<0x114, 0xf>(v);
    v = dpp_add<0x118, 0xf>(v);
    v = dpp_add<0x142, 0xa>(v);
    v = dpp_add<0x143, 0xc>(v);
    return v;
}
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t& total)
{
    const uint32_t inc = wave_incl_scan(v);
    total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    return inc - v;
}

template <int NT>
__global__ __launch_bounds__(256) void k_ii_fill_w(const uint8_t* __restrict__ frames, int pitch,
                                                   long long fstride, int W, int H, int nbands,
                                                   const uint32_t* __restrict__ colpre, int CW,
                                                   int32_t* __restrict__ ii, int ip, long long istride, int nframes,
                                                   int br)
{
    const int gw = blockIdx.x * 4 + (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int f = gw / nbands, band = gw - f * nbands;
    if (f >= nframes) return;
    const int lane = (int)lane_id();
    const int y0 = band * br;
    const int rows = min(br, H - y0);
    // acc = ii[y0][x]: exclusive row scan of the column sums above the band
    uint32_t acc[NT][4];
    {
        const uint32_t* c = colpre + ((size_t)f * nbands + band) * CW;
        uint32_t carry = 0u;
#pragma unroll
        for (int t = 0; t < NT; t++) {
            const int x = 4 * lane + 256 * t;
            uint32_t v[4];
#pragma unroll
            for (int j = 0; j < 4; j++) v[j] = (x + j < W) ? c[x + j] : 0u;
            const uint32_t e1 = v[0], e2 = e1 + v[1], e3 = e2 + v[2], tot = e3 + v[3];
            uint32_t wt;
            const uint32_t base = carry + wave_excl_scan(tot, wt);
            carry += wt;
            acc[t][0] = base; acc[t][1] = base + e1; acc[t][2] = base + e2; acc[t][3] = base + e3;
        }
    }
    uint32_t* out = reinterpret_cast<uint32_t*>(ii) + (size_t)f * istride;
    if (band == 0) {
#pragma unroll
        for (int t = 0; t < NT; t++) {
            const int x = 4 * lane + 256 * t;
            if (x < ip) *reinterpret_cast<uint4*>(out + x) = make_uint4(0u, 0u, 0u, 0u);
        }
    }
    const uint8_t* src = frames + (size_t)f * fstride + (size_t)y0 * pitch;
    // the band's pixel rows stream through a ring of kFillAhead rows loaded
    // ahead (the row scan no longer waits a memory latency per row: a single
    // frame's 34 band waves were latency-bound)
    constexpr int kFillAhead = 4;
    uint32_t wq[kFillAhead][NT];
    auto ldrow = [&](int r, uint32_t (&wv)[NT]) {
        const uint8_t* row = src + (size_t)min(r, rows - 1) * pitch;     // past the band: a repeat, unused
#pragma unroll
        for (int t = 0; t < NT; t++) {
            const int x = 4 * lane + 256 * t;
            wv[t] = (x + 4 <= pitch) ? *reinterpret_cast<const uint32_t*>(row + x) : 0u;
        }
    };
    static_for<kFillAhead>([&](auto dc) { ldrow(decltype(dc)::value, wq[decltype(dc)::value]); });
    for (int r0 = 0; r0 < rows; r0 += kFillAhead) {
        static_for<kFillAhead>([&](auto dc) {
            constexpr int D = decltype(dc)::value;
            const int r = r0 + D;
            if (r >= rows) return;
            uint32_t wv[NT];
#pragma unroll
            for (int t = 0; t < NT; t++) wv[t] = wq[D][t];
            ldrow(r + kFillAhead, wq[D]);
            uint32_t* dst = out + (size_t)(y0 + r + 1) * ip;
            uint32_t carry = 0u;
#pragma unroll
            for (int t = 0; t < NT; t++) {
                const int x = 4 * lane + 256 * t;
                uint32_t p[4];
#pragma unroll
                for (int j = 0; j < 4; j++) p[j] = (x + j < W) ? (wv[t] >> (8 * j)) & 0xffu : 0u;
                const uint32_t e1 = p[0], e2 = e1 + p[1], e3 = e2 + p[2], tot = e3 + p[3];
                uint32_t wt;
                const uint32_t base = carry + wave_excl_scan(tot, wt);
                carry += wt;
                acc[t][0] += base; acc[t][1] += base + e1; acc[t][2] += base + e2; acc[t][3] += base + e3;
                // pad columns (> W) stay zero (set once at detector creation and
                // never written: 6 % of the 1080p row): the flat reads of
                // getTrace can land on them
                if (x <= W) {
                    const uint4 o4 = make_uint4(x <= W ? acc[t][0] : 0u, x + 1 <= W ? acc[t][1] : 0u,
                                                x + 2 <= W ? acc[t][2] : 0u, x + 3 <= W ? acc[t][3] : 0u);
                    // nontemporal: the 2.3-GB batch integral streams past the
                    // caches (whole step 5.21 -> 5.19 ms, 3 A/B pairs)
                    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                    __builtin_nontemporal_store(u32x4{o4.x, o4.y, o4.z, o4.w}, reinterpret_cast<u32x4*>(dst + x));
                }
            }
        });
    }
}

static void launch_bandscan(uint32_t* colsum, int nbands, int CW, int W, int nframes, hipStream_t s)
{
    if (nbands <= 48) k_ii_bandscan<48><<<dim3((W + 255) / 256, nframes), 256, 0, s>>>(colsum, nbands, CW, W);
    else if (nbands <= 136) k_ii_bandscan<136><<<dim3((W + 255) / 256, nframes), 256, 0, s>>>(colsum, nbands, CW, W);
    else k_ii_bandscan<272><<<dim3((W + 255) / 256, nframes), 256, 0, s>>>(colsum, nbands, CW, W);
}

hipError_t launch_integral(const uint8_t* frames, int pitch, long long fstride, int nframes,
                           const FrameParams& P, uint32_t* colsum, int32_t* ii, hipStream_t s)
{
    // small batches: 8-row bands (4x the band waves of the fill pass, which
    // is one wave per band) -- colsum is sized for both (integral_bands())
    const int br = nframes <= kSmallBatch ? small_band_rows() : big_band_rows();
    const int nbands = (P.H + br - 1) / br;
    const int W = P.W;
    dim3 grid(nbands, nframes);
    if (W + 1 <= 2048) {
        const int CW = 2048;
        k_ii_bandsum<8><<<grid, 256, 0, s>>>(frames, pitch, fstride, W, P.H, nbands, colsum, CW, br);
        launch_bandscan(colsum, nbands, CW, W, nframes, s);
        k_ii_fill_w<8><<<(nbands * nframes + 3) / 4, 256, 0, s>>>(frames, pitch, fstride, W, P.H, nbands, colsum, CW,
                                                                    ii, P.ip, P.ii_stride, nframes, br);
    } else if (W + 1 <= 4096) {
        const int CW = 4096;
        k_ii_bandsum<16><<<grid, 256, 0, s>>>(frames, pitch, fstride, W, P.H, nbands, colsum, CW, br);
        launch_bandscan(colsum, nbands, CW, W, nframes, s);
        k_ii_fill_w<16><<<(nbands * nframes + 3) / 4, 256, 0, s>>>(frames, pitch, fstride, W, P.H, nbands, colsum,
                                                                     CW, ii, P.ip, P.ii_stride, nframes, br);
    } else if (W + 1 <= 8192) {
        // wide frames (up to 8,191 columns): 32 columns per thread, the
        // workgroup-scan fill (one 256-thread block per band, two barriers a row)
        const int CW = 8192;
        k_ii_bandsum<32><<<grid, 256, 0, s>>>(frames, pitch, fstride, W, P.H, nbands, colsum, CW, br);
        launch_bandscan(colsum, nbands, CW, W, nframes, s);
        k_ii_fill<32><<<grid, 256, 0, s>>>(frames, pitch, fstride, W, P.H, nbands, colsum, CW, ii, P.ip, P.ii_stride,
                                           br);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ======================================================================
// Hessian determinant (calcHessianMultiConst, surfd.cu:445-481; getHessian
// surfd.cu:353-366).  One thread per response sample of one octave, all
// scales of the octave; cells outside a scale's valid window are written 0
// (the reference's cudaMemset, surf.cpp:348).  Planes 0/1 of octaves > 0
// (the reference's halfImage copies, surfd.cu:321-331) are never
// materialised: k_nms reads them from the previous octave's planes 2/4.
// ======================================================================

// getSum (surfd.cu:334-343): inclusive rect [x2..x1] x [y2..y1].
__device__ __forceinline__ uint32_t box(const uint32_t* __restrict__ I, int ip, int x1, int y1, int x2, int y2)
{
    const int yp1 = (y1 + 1) * ip;
    const int yp2 = y2 * ip;
    return I[yp1 + x1 + 1] + I[yp2 + x2] - I[yp2 + x1 + 1] - I[yp1 + x2];
}

__device__ __forceinline__ float hessian_at(const uint32_t* __restrict__ I, int ip, int x0, int y0,
                                            int m, int x2, int x3, int x4)
{
    const int xp = x0 + m, xm = x0 - m, yp = y0 + m, ym = y0 - m;
    const int32_t sxx = (int32_t)(box(I, ip, xp + x2, y0 + x3, xm - x2, y0 - x3)
                                  - 3u * box(I, ip, x0 + x2, y0 + x3, x0 - x2, y0 - x3));
    const int32_t syy = (int32_t)(box(I, ip, x0 + x3, yp + x2, x0 - x3, ym - x2)
                                  - 3u * box(I, ip, x0 + x3, y0 + x2, x0 - x3, y0 - x2));
    const int32_t sxy = (int32_t)(box(I, ip, x0 + x4, y0, x0, y0 - x4)
                                  + box(I, ip, x0, y0 + x4, x0 - x4, y0)
                                  - box(I, ip, x0 + x4, y0 + x4, x0, y0)
                                  - box(I, ip, x0, y0, x0 - x4, y0 - x4));
    const float rr = INV255 * INV255;
    const float dxx = (float)sxx;
    const float dyy = (float)syy;
    const float dxy = 0.6f * (float)sxy;
    const float a = dxx * dyy;
    const float b = dxy * dxy;
    return rr * (a - b);
}

#include "surfhip_hess_q0.inc"
#include "surfhip_hess_q1.inc"
#include "surfhip_hess_p0.inc"
#include "surfhip_hess_w.inc"

// The row sums the integral writer's strips add to their local integral
// (plan.iiw): strip k's local integral starts at its halo column cs_k = ST k
// - HALO (k_hess_w: 480 k - 144; k_hess_p0: 128 k - 16), so the image's
// integral is L_k(R, c) + II(R, cs_k), and II(R, cs_k) is the running sum
// over pixel rows r < R of S_k(r) = the sum of row r over columns [0, cs_k).
// One wave per pixel row: a wave scan of the row's dword sums, chunk by chunk
// with a running carry; the lane holding the last dword before cs_k stores
// S_k(r).  Reads columns [0, cs_{ns-1}) of the frame once (1,296 of 1,920 at
// 1080p for k_hess_w's strips).
// (16 VGPRs: its waves fit beside k_describe_u2's, which leave 20 of a SIMD
// lane's 512 free, so the pass of the next batch runs inside describe)
template <int ST, int HALO>
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(16))) void k_ii_rowseg(
    const uint8_t* __restrict__ frames, int pitch, long long fstride, int H, int ns, int rs_rows,
    uint32_t* __restrict__ rowseg)
{
    static_assert(ST % 4 == 0 && HALO % 4 == 0, "strip boundaries on dword boundaries");
    const int f = blockIdx.y;
    const int r = blockIdx.x * 4 + (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (r >= H) return;
    const int lane = (int)lane_id();
    const int nd = (ST * (ns - 1) - HALO) / 4;                // dwords below the last boundary
    // the row's dwords [0, nd): a buffer load past them returns 0
    const rsrc_t R = make_rsrc(frames + (size_t)f * fstride + (size_t)r * pitch, (long long)nd * 4);
    uint32_t* out = rowseg + (size_t)f * ns * rs_rows + r;
    uint32_t carry = 0u;
    constexpr int KC = 6;                                      // loads in flight per lane
    for (int d0 = 0; d0 < nd; d0 += 64 * KC) {
        uint32_t v[KC];
#pragma unroll
        for (int i = 0; i < KC; i++)
            v[i] = __builtin_amdgcn_raw_buffer_load_b32(R, (uint32_t)(d0 + 64 * i + lane) * 4u, 0, 0);
#pragma unroll
        for (int i = 0; i < KC; i++) {
            const int d = d0 + 64 * i + lane;
            const uint32_t x = __builtin_amdgcn_udot4(v[i], 0x01010101u, 0u, false);
            uint32_t tot;
            const uint32_t inc = carry + wave_excl_scan(x, tot) + x;
            carry += tot;
            // dword d ends at column 4 d + 3: the last one below cs_k when
            // 4 (d + 1) = ST k - HALO, i.e. d + 1 + HALO / 4 = (ST / 4) k
            constexpr int DO = 1 + HALO / 4;
            if (d < nd && (d + DO) % (ST / 4) == 0) out[(size_t)((d + DO) / (ST / 4)) * rs_rows] = inc;
        }
    }
}

hipError_t launch_rowseg(const uint8_t* frames, int pitch, long long fstride, int nframes, const FrameParams& P,
                         const LaunchPlan& plan, uint32_t* rowseg, hipStream_t s)
{
    if (!plan.iiw || plan.rs_nstrips < 2) return hipSuccess;
    const dim3 g((P.H + 3) / 4, nframes);
    if (plan.iiw == 2)
        k_ii_rowseg<128, 16><<<g, 256, 0, s>>>(frames, pitch, fstride, P.H, plan.rs_nstrips, plan.rs_rows, rowseg);
    else
        k_ii_rowseg<hw::ST, hw::H><<<g, 256, 0, s>>>(frames, pitch, fstride, P.H, plan.rs_nstrips, plan.rs_rows,
                                                     rowseg);
    return hipGetLastError();
}

// Octave 1 on k_hess_q1 (only when k_hess_w is off: 2-octave detectors or
// SURFHIP_HESS_W=0) needs the geometry compiled into it (sampling 2, lobes
// 15/19/23).
static bool q1_ok(const FrameParams& P, const OctaveParams& q)
{
    static const int masks[3] = {15, 19, 23};
    if (P.sampling != 2 || q.delta != 4 || q.nscale != 3 || q.init_scale != 2) return false;
    for (int i = 0; i < 3; i++)
        if (q.mask[i] != masks[i] || q.x2[i] != masks[i] / 2 || q.x3[i] != 2 * (masks[i] / 2) ||
            q.x4[i] != 3 * (masks[i] / 2))
            return false;
    return true;
}

// Octave 0 on k_hess_q0 when its geometry is the one compiled into it
// (sampling 2, lobes 3/5/7/9/11).
static bool q0_ok(const FrameParams& P, const OctaveParams& q)
{
    static const int masks[5] = {3, 5, 7, 9, 11};
    if (P.sampling != 2 || q.delta != 2 || q.nscale != 5 || q.init_scale != 0) return false;
    for (int i = 0; i < 5; i++)
        if (q.mask[i] != masks[i] || q.x2[i] != masks[i] / 2 || q.x3[i] != 2 * (masks[i] / 2) ||
            q.x4[i] != 3 * (masks[i] / 2))
            return false;
    return true;
}

// k_hessian_t0 (octave 0 of the gather plan from LDS tiles): sample rows per
// workgroup and the corners' reach it stages (16 for init mask 9: lobe 11,
// m + x2 = 16)
constexpr int kT0BY = 8;
constexpr int kT0Halo = 16;

// Octaves 1 .. n of the default geometry (sampling 2, init mask 9: lobes
// 15/19/23, 31/39/47, 63/79/95) on k_hess_w; returns n (2 or 3) or 0.
static int hw_octaves(const FrameParams& P, const OctaveParams* oct)
{
    if (P.sampling != 2 || P.noct < 3) return 0;
    int n = 0;
    for (int o = 1; o <= 3 && o < P.noct; o++) {
        const OctaveParams& q = oct[o];
        bool ok = q.delta == (2 << o) && q.nscale == 3 && q.init_scale == 2;
        for (int i = 0; ok && i < 3; i++) {
            const int K = hw::kof(o, i);
            ok = q.mask[i] == 2 * K + 1 && q.x2[i] == K && q.x3[i] == 2 * K && q.x4[i] == 3 * K;
        }
        if (!ok) break;
        n = o;
    }
    return n >= 2 ? n : 0;
}

// Which kernel computes each octave's planes:
//   octave 0      k_hess_q0 (u8 frame; default geometry, batches > kGatherBatch)
//   octaves 1-3   k_hess_w (u8 frame; default geometry, 3+ octaves)
//   octave 1      k_hess_q1 when k_hess_w is off (2 octaves, or SURFHIP_HESS_W=0);
//                 k_hess_q0 + k_hess_q1 in one launch (k_hess_q01) unless SURFHIP_Q01=0
//   the rest      k_hessian, one thread per sample over the integral image
//                 (every octave for batches <= kGatherBatch or SURFHIP_HESS_GATHER=1)
void make_plan(const FrameParams& P, const OctaveParams* oct, LaunchPlan& plan, int max_batch)
{
    plan = LaunchPlan{};
    int hb = 0, nb = 0;
    const char* ge = getenv("SURFHIP_HESS_GATHER");
    const bool gather = ge ? atoi(ge) != 0 : max_batch <= kGatherBatch;
    const char* we = getenv("SURFHIP_HESS_W");
    plan.hw_n = (!gather && !(we && atoi(we) == 0)) ? hw_octaves(P, oct) : 0;
    plan.hw_nstrips = (P.W + hw::ST - 1) / hw::ST;
    plan.hw_nblk = ((P.H / 4 + 1 + hw::U - 1) / hw::U) * hw::U;
    plan.q0 = !gather && P.noct > 0 && q0_ok(P, oct[0]);
    plan.q0_strips = (oct[0].sw + 63) / 64;
    plan.q1 = !gather && P.noct > 1 && plan.hw_n == 0 && q1_ok(P, oct[1]);
    plan.q1_strips = P.noct > 1 ? (oct[1].sw + 63) / 64 : 0;
    const char* me = getenv("SURFHIP_Q01");
    plan.q01 = plan.q0 && plan.q1 && !(me && atoi(me) == 0);
    // octave 0 on k_hess_p0 unless SURFHIP_P0=0; SURFHIP_P0=BG picks its
    // barrier interval B (steps) and consumer waves G
    // (value 10 B + G: barrier interval B steps, G consumer waves)
    const char* pe = getenv("SURFHIP_P0");
    plan.p0 = (plan.q0 && !plan.q01) ? (pe ? atoi(pe) : 93) : 0;
    if (plan.p0 != 0 && plan.p0 != 95 && plan.p0 != 94 && plan.p0 != 93 && plan.p0 != 92 && plan.p0 != 91 &&
        plan.p0 != 32 && plan.p0 != 33)
        plan.p0 = 93;
    // the gather plan's octave 0 from LDS tiles (k_hessian_t0) when its
    // corners reach at most kT0Halo integral samples from the sample and the
    // sampling step is 2 (the default geometry); SURFHIP_HESS_T0=0 disables
    {
        const char* te = getenv("SURFHIP_HESS_T0");
        const OctaveParams& q = oct[0];
        int reach = 0;
        for (int i = 0; i < q.nscale; i++) reach = std::max(reach, std::max(q.mask[i] + q.x2[i], q.x4[i]));
        plan.t0 = gather && P.noct > 0 && q.delta == 2 && reach <= kT0Halo && !(te && atoi(te) == 0);
        plan.t0_nbx = (q.sw + 63) / 64;
        plan.t0_nby = (q.sh + kT0BY - 1) / kT0BY;
    }
    for (int o = 0; o < kMaxOct; o++) {
        plan.hess_start[o] = hb;
        plan.nms_start[o] = nb;
        if (o < P.noct) {
            const OctaveParams& q = oct[o];
            plan.hess_nbx[o] = (q.sw + 63) / 64;
            const bool on_u8 = (o == 0 && plan.q0) || (o == 1 && plan.q1) || (o >= 1 && o <= plan.hw_n);
            if (!on_u8 && !(o == 0 && plan.t0)) hb += plan.hess_nbx[o] * ((q.sh + 3) / 4);
            plan.nms_nbx[o] = (q.nms_gx + 63) / 64;
            plan.nms_nby[o] = (q.nms_gy + kScanRows - 1) / kScanRows;
            nb += ((P.max_scale - 1) / 2) * plan.nms_nbx[o] * plan.nms_nby[o];   // levels k = 1, 3, .. < max_scale - 1
        } else {
            plan.hess_nbx[o] = plan.nms_nbx[o] = plan.nms_nby[o] = 1;
        }
    }
    plan.hess_start[kMaxOct] = hb;
    plan.nms_start[kMaxOct] = nb;
    // the integral image from k_hess_w (SURFHIP_II_FUSE=0 disables, =2 moves
    // it to k_hess_p0's producer): octave 0 on k_hess_p0 and octaves 1-3 on
    // k_hess_w; octaves past 3 (k_hessian) then read the integral written,
    // after them on the same stream
    {
        const char* fe = getenv("SURFHIP_II_FUSE");
        const int fv = fe ? atoi(fe) : 1;
        const bool on = plan.hw_n >= 2 && plan.p0 != 0 && !plan.t0 && fv != 0;
        plan.iiw = !on ? 0 : (fv == 2 && plan.p0 == 93) ? 2 : 1;
        plan.rs_rows = 4 * plan.hw_nblk;
        plan.rs_nstrips = plan.iiw == 2 ? plan.q0_strips : plan.hw_nstrips;
    }
}

std::string hessian_plan_text(const LaunchPlan& plan, const FrameParams& P)
{
    std::string t;
    auto add = [&](const char* k, int o0, int o1) {
        if (o1 < o0) return;
        if (!t.empty()) t += " + ";
        t += k;
        t += o0 == o1 ? " (octave " + std::to_string(o0) + ")"
                      : " (octaves " + std::to_string(o0) + "-" + std::to_string(o1) + ")";
    };
    if (plan.q01) {
        add("k_hess_q01", 0, 1);
    } else {
        if (plan.p0) add("k_hess_p0", 0, 0);
        else if (plan.q0) add("k_hess_q0", 0, 0);
        if (plan.q1) add("k_hess_q1", 1, 1);
    }
    if (plan.t0) add("k_hessian_t0", 0, 0);
    if (plan.hw_n > 0) add("k_hess_w", 1, plan.hw_n);
    // (the row-sum pass runs before the stage: beside the previous batch's
    // NMS when pipelined, like the integral passes it replaces)
    if (plan.iiw) t += plan.iiw == 2 ? ", writing the integral image (k_hess_p0)" : ", writing the integral image";
    if (plan.hess_start[kMaxOct] > 0) {
        int lo = -1, hi = -1;
        for (int o = 0; o < P.noct; o++)
            if (plan.hess_start[o + 1] > plan.hess_start[o]) { if (lo < 0) lo = o; hi = o; }
        if (lo >= 0) add("k_hessian", lo, hi);
    }
    return t;
}

__device__ __forceinline__ int octave_of(const int* start, int noct, int b)
{
    int o = 0;
    while (o + 1 < noct && b >= start[o + 1]) o++;
    return o;
}

// 1-D grid of nf8 * per workgroups, XCD-aware: the workgroups of XCD x
// (blockIdx % 8) take frames x, x + 8, ..., each frame's `per` workgroups
// together, so a frame's integral image / response planes are fetched into
// one XCD's L2 instead of all eight.
// Batches of fewer than 8 frames spread each frame's workgroups over all
// XCDs instead (one frame per XCD would leave the others idle); the grid is
// frame_grid(nframes) * per.
__device__ __forceinline__ bool xcd_frame_block(int per, int nframes, int& f, int& lb)
{
    if (nframes < 8) {
        f = blockIdx.x / per;
        lb = blockIdx.x - f * per;
        return f < nframes;
    }
    const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
    f = (k / per) * 8 + xcd;
    lb = k - (k / per) * per;
    return f < nframes;
}
static inline int frame_grid(int nframes) { return nframes < 8 ? nframes : (nframes + 7) & ~7; }

// All octaves (not on an LDS ring) of a frame in one launch: the local block
// index walks the octaves' sample grids (64 x 4 samples per block).
__global__ __launch_bounds__(256) void k_hessian(const int32_t* __restrict__ ii, float* __restrict__ resp,
                                                 FrameParams P, const OctaveParams* __restrict__ oct,
                                                 LaunchPlan plan, int nframes)
{
    int f, gb;
    if (!xcd_frame_block(plan.hess_start[kMaxOct], nframes, f, gb)) return;
    const int o = octave_of(plan.hess_start, P.noct, gb);
    const OctaveParams& q = oct[o];
    const int lb = gb - plan.hess_start[o];
    const int nbx = plan.hess_nbx[o];
    const int ix = (lb % nbx) * 64 + (threadIdx.x & 63);
    const int iy = (lb / nbx) * 4 + (threadIdx.x >> 6);
    if (ix >= q.sw || iy >= q.sh) return;
    const uint32_t* I = reinterpret_cast<const uint32_t*>(ii) + (size_t)f * P.ii_stride;
    float* R = resp + (size_t)f * P.resp_stride + q.ooff + (size_t)iy * q.sp + ix;
    const int x0 = q.delta * ix, y0 = q.delta * iy;
    const int ns = q.nscale;
#pragma unroll
    for (int i = 0; i < kMaxScale; i++) {
        if (i >= ns) break;
        const int b1 = q.b1[i];
        float v = 0.f;
        if (ix >= b1 && ix < q.sw - b1 && iy >= b1 && iy < q.sh - b1)
            v = hessian_at(I, P.ip, x0, y0, q.mask[i], q.x2[i], q.x3[i], q.x4[i]) * q.norm[i];
        R[(size_t)(q.init_scale + i) * q.osize] = v;
    }
}

// Octave 0 of the gather plan (few frames, config #2) from LDS tiles: a
// workgroup loads the integral-image tile under its 64 x kT0BY samples (the
// samples' span plus every corner's reach, kT0Halo on each side) with
// coalesced row loads, then each thread computes its samples' scales with
// hessian_at reading the tile -- the 32 corners of a response are LDS reads
// instead of global gathers (k_hessian: 32 dependent-latency gathers per
// response, 55 us for one 1080p frame's four octaves, 80 % of the responses
// in octave 0).  Same integer box sums and float ops as k_hessian, so the
// planes are bit-identical.
template <int HALO>
__global__ __launch_bounds__(256) void k_hessian_t0(const int32_t* __restrict__ ii, float* __restrict__ resp,
                                                    FrameParams P, OctaveParams q, int nbx, int nby, int nframes)
{
    constexpr int TW = 2 * 63 + 2 * HALO + 2;           // tile columns: integral x in [2 ix0 - HALO, ..]
    constexpr int TH = 2 * (kT0BY - 1) + 2 * HALO + 2;  // tile rows
    __shared__ uint32_t T[TH * TW];
    int f, lb;
    if (!xcd_frame_block(nbx * nby, nframes, f, lb)) return;
    const int by = lb / nbx, bx = lb - by * nbx;
    const int ix0 = bx * 64, iy0 = by * kT0BY;
    const int tx0 = 2 * ix0 - HALO, ty0 = 2 * iy0 - HALO;
    const uint32_t* I = reinterpret_cast<const uint32_t*>(ii) + (size_t)f * P.ii_stride;
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    // rows by wave, columns by lane (coalesced); coordinates outside the
    // image are clamped -- only samples outside the borders, which are not
    // computed, would read them
    for (int r = wv; r < TH; r += 4) {
        const int gy = min(max(ty0 + r, 0), P.iH - 1);
        const uint32_t* row = I + (size_t)gy * P.ip;
#pragma unroll
        for (int c0 = 0; c0 < TW; c0 += 64) {
            const int c = c0 + lane;
            if (c < TW) T[r * TW + c] = row[min(max(tx0 + c, 0), P.ip - 1)];
        }
    }
    __syncthreads();
    const int ix = ix0 + lane;
    for (int k = wv; k < kT0BY; k += 4) {
        const int iy = iy0 + k;
        if (ix >= q.sw || iy >= q.sh) continue;
        float* R = resp + (size_t)f * P.resp_stride + q.ooff + (size_t)iy * q.sp + ix;
        const int lx = 2 * lane + HALO, ly = 2 * k + HALO;          // (x0, y0) in the tile
#pragma unroll
        for (int i = 0; i < kMaxScale; i++) {
            if (i >= q.nscale) break;
            const int b1 = q.b1[i];
            float v = 0.f;
            if (ix >= b1 && ix < q.sw - b1 && iy >= b1 && iy < q.sh - b1)
                v = hessian_at(T, TW, lx, ly, q.mask[i], q.x2[i], q.x3[i], q.x4[i]) * q.norm[i];
            R[(size_t)(q.init_scale + i) * q.osize] = v;
        }
    }
}

hipError_t launch_hessian(const uint8_t* frames, int pitch, long long fstride, const int32_t* ii, float* resp,
                          int nframes, const FrameParams& P, const OctaveParams* d_oct, const OctaveParams* h_oct,
                          const LaunchPlan& plan, hipStream_t s, int parts, const uint32_t* rowseg, int32_t* ii_out)
{
    const int nf8 = (nframes + 7) & ~7;
    // parts: 1 = the kernels that read the u8 frames, 2 = those that read the
    // integral image (the two may run on different streams)
    // (4 / 8: only the octave-0 / only the k_hess_w launch of part 1)
    const bool p0p = (parts & 5) != 0, wp = (parts & 9) != 0, iip = (parts & 2) != 0;
    const bool u8p = p0p || wp;
    if (u8p && !frames && (plan.q0 || plan.q1 || plan.hw_n > 0)) return hipErrorInvalidValue;
    auto launch_w = [&]() {
        if (plan.hw_n > 0) {
            const dim3 g(nf8 * plan.hw_nstrips);
            const OctaveParams& q3 = h_oct[plan.hw_n >= 3 ? 3 : 2];
            const bool wr = plan.iiw == 1 && ii_out && rowseg;
#define HW_LAUNCH(NO, IIW)                                                                                       \
    k_hess_w<NO, IIW><<<g, hw::THREADS, 0, s>>>(frames, pitch, fstride, resp, P, h_oct[1], h_oct[2], q3,          \
                                                plan.hw_nstrips, nframes, plan.hw_nblk, rowseg, ii_out, plan.rs_rows)
            if (plan.hw_n >= 3) {
                if (wr) HW_LAUNCH(3, true);
                else HW_LAUNCH(3, false);
            } else {
                if (wr) HW_LAUNCH(2, true);
                else HW_LAUNCH(2, false);
            }
#undef HW_LAUNCH
        }
    };
    if (p0p) {
        const int nb0 = 8 * (((nf8 / 8) * plan.q0_strips + q0::WAVES - 1) / q0::WAVES);
        const int nb1 = 8 * (((nf8 / 8) * plan.q1_strips + q1::WAVES - 1) / q1::WAVES);
        if (plan.q01) {
            k_hess_q01<<<dim3(nb0 + nb1), q0::THREADS, 0, s>>>(frames, pitch, fstride, resp, P, h_oct[0], h_oct[1],
                                                               plan.q0_strips, plan.q1_strips, nb0, nframes);
        } else {
            const dim3 gp(nf8 * plan.q0_strips);
            const int pb = plan.p0 / 10, pg = plan.p0 % 10;      // interval, consumer waves
            // (iiw 2, only with the default 93: this launch writes the integral)
            const bool wr0 = plan.iiw == 2 && ii_out && rowseg;
#define P0_CASE(BB, GG)                                                                                          \
    else if (pb == BB && pg == GG) k_hess_p0<BB, GG, SURF_P0_PLANE_NT, false><<<gp, 64 * (1 + GG), 0, s>>>(        \
        frames, pitch, fstride, resp, P, h_oct[0], plan.q0_strips, nframes, nullptr, nullptr, 0);
            if (wr0 && pb == 9 && pg == 3)
                k_hess_p0<9, 3, SURF_P0_PLANE_NT, true><<<gp, 64 * 4, 0, s>>>(frames, pitch, fstride, resp, P, h_oct[0],
                                                               plan.q0_strips, nframes, rowseg, ii_out, plan.rs_rows);
            P0_CASE(9, 5) P0_CASE(9, 4) P0_CASE(9, 3) P0_CASE(9, 2) P0_CASE(9, 1) P0_CASE(3, 2) P0_CASE(3, 3)
#undef P0_CASE
            else if (plan.q0)
                k_hess_q0<4, 1, 2><<<dim3(nb0), q0::THREADS, 0, s>>>(frames, pitch, fstride, resp, P, h_oct[0],
                                                                     plan.q0_strips, nframes);
            if (plan.q1)
                k_hess_q1<2><<<dim3(nb1), q1::THREADS, 0, s>>>(frames, pitch, fstride, resp, P, h_oct[1],
                                                               plan.q1_strips, nframes);
        }
    }
    if (wp) launch_w();
    if (plan.t0 && iip)
        k_hessian_t0<kT0Halo><<<dim3(frame_grid(nframes) * plan.t0_nbx * plan.t0_nby), 256, 0, s>>>(
            ii, resp, P, h_oct[0], plan.t0_nbx, plan.t0_nby, nframes);
    if (plan.hess_start[kMaxOct] > 0 && iip)
        k_hessian<<<dim3(frame_grid(nframes) * plan.hess_start[kMaxOct]), 256, 0, s>>>(ii, resp, P, d_oct, plan,
                                                                                        nframes);
    return hipGetLastError();
}

// ======================================================================
// Scale-space NMS + interpolation + makePoint (findMaximumWithInterp,
// surfd.cu:676-832; fitQuadrat 942-988; solveLinearSystem 835-887;
// makePoint 1001-1022).  One thread per 2x2 block of one NMS level.
// Survivors are compacted per wave (ballot + one atomic per wave) into the
// frame's candidate buffer with a canonical key (octave, level, row, col);
// k_sort restores that order, so the output is deterministic.
// ======================================================================

__device__ void solve3(float* sol, float (&sq)[3][3])
{
    int row, col, c, pivot = 0, i;
    float maxc, coef, temp, mult, val;
    for (col = 0; col < 2; col++) {
        maxc = -1.f;
        for (row = col; row < 3; row++) {
            coef = sq[row][col];
            coef = (coef < 0.f ? -coef : coef);
            if (coef > maxc) { maxc = coef; pivot = row; }
        }
        if (pivot != col) {
            for (i = 0; i < 3; i++) { temp = sq[pivot][i]; sq[pivot][i] = sq[col][i]; sq[col][i] = temp; }
            temp = sol[pivot]; sol[pivot] = sol[col]; sol[col] = temp;
        }
        for (row = col + 1; row < 3; row++) {
            mult = sq[row][col] / sq[col][col];
            for (c = col; c < 3; c++) sq[row][c] = sq[row][c] - mult * sq[col][c];
            sol[row] = sol[row] - mult * sol[col];
        }
    }
    for (row = 2; row >= 0; row--) {
        val = sol[row];
        for (col = 2; col > row; col--) val = val - sol[col] * sq[row][col];
        sol[row] = val / sq[row][row];
    }
}

// Response planes of one octave as the reference lays them out after its
// halfImage copies: planes 0/1 of octave o > 0 are read in place from octave
// o-1's planes 2/4 at (2r, 2c), which is exactly what halfImage copied.
struct OctView {
    const float* F;                 // the frame's response block
    int cur;                        // float offset of this octave's plane 0
    int sp, osize;
    int half;                       // octave > 0: planes 0 / 1 are the halfImage views
    // plane 0's view and plane 1's differences from it (a select against a
    // constant: selecting between two fields became a select of their
    // addresses and put the view in scratch)
    int hb, hr, hc, dhb, dhr, dhc;
    // branch-free (selects): a branch around a load makes hipcc wait for the
    // loads issued before it at the join, which serialised the NMS scan's 32
    // block loads into 16 memory round trips
    __device__ __forceinline__ int off(int s, int r, int c) const
    {
        const bool h = half && s < 2;
        const bool p1 = s != 0;
        const int base = h ? hb + (p1 ? dhb : 0) : cur + s * osize;
        return base + r * (h ? hr + (p1 ? dhr : 0) : sp) + c * (h ? hc + (p1 ? dhc : 0) : 1);
    }
    __device__ __forceinline__ float operator()(int s, int r, int c) const { return F[off(s, r, c)]; }
    // (s, r, c) and (s, r, c + 1) of a plane that is not a halfImage view:
    // one 8-byte load (4-byte aligned)
    __device__ __forceinline__ void pair_full(int s, int r, int c, float& a, float& b) const
    {
        typedef float f2a4 __attribute__((ext_vector_type(2), aligned(4)));
        const f2a4 v = *reinterpret_cast<const f2a4*>(F + cur + s * osize + r * sp + c);
        a = v.x;
        b = v.y;
    }
    // (s, r, c) and (s, r, c + 1)
    __device__ __forceinline__ void pair(int s, int r, int c, float& a, float& b) const
    {
        const bool h = half && s < 2;
        const int o = off(s, r, c);
        a = F[o];
        b = F[o + (h ? hc + (s != 0 ? dhc : 0) : 1)];
    }
};

// fitQuadrat (surfd.cu:942-988) on the 19 responses it reads around (s, r,
// c): v = {c, s+1, s-1, r+1, r-1, c+1, c-1, (s+1, r+1), (s+1, r-1),
// (s-1, r+1), (s-1, r-1), (s+1, c+1), (s+1, c-1), (s-1, c+1), (s-1, c-1),
// (r+1, c+1), (r+1, c-1), (r-1, c+1), (r-1, c-1)} (the NMS scan writes this
// record for its survivors, k_nms_scan)
__device__ float fit_quad_v(const float* v, float (&off)[3])
{
    const float c0 = v[0];
    const float nx0 = v[1], pv0 = v[2];
    const float cnr = v[3], cpr = v[4], cnc = v[5], cpc = v[6];
    float g[3], H[3][3];
    g[0] = (nx0 - pv0) * 0.5f;
    g[1] = (cnr - cpr) * 0.5f;
    g[2] = (cnc - cpc) * 0.5f;
    const float temp = c0 + c0;
    H[0][0] = (pv0 + nx0) - temp;
    H[1][1] = (cnr + cpr) - temp;
    H[2][2] = (cnc + cpc) - temp;
    H[0][1] = ((v[7] - v[8]) - (v[9] - v[10])) * 0.25f;
    H[0][2] = ((v[11] - v[12]) - (v[13] - v[14])) * 0.25f;
    H[1][2] = ((v[15] - v[16]) - (v[17] - v[18])) * 0.25f;
    H[1][0] = H[0][1];
    H[2][0] = H[0][2];
    H[2][1] = H[1][2];
    off[0] = -g[0];
    off[1] = -g[1];
    off[2] = -g[2];
    solve3(off, H);
    const float dot = (off[0] * g[0] + off[1] * g[1]) + off[2] * g[2];
    return c0 + 0.5f * dot;
}

__device__ float fit_quad(const OctView& V, float (&off)[3], int s, int r, int c)
{
    const float v[19] = {V(s, r, c),
                         V(s + 1, r, c),         V(s - 1, r, c),
                         V(s, r + 1, c),         V(s, r - 1, c),
                         V(s, r, c + 1),         V(s, r, c - 1),
                         V(s + 1, r + 1, c),     V(s + 1, r - 1, c),     V(s - 1, r + 1, c),     V(s - 1, r - 1, c),
                         V(s + 1, r, c + 1),     V(s + 1, r, c - 1),     V(s - 1, r, c + 1),     V(s - 1, r, c - 1),
                         V(s, r + 1, c + 1),     V(s, r + 1, c - 1),     V(s, r - 1, c + 1),     V(s, r - 1, c - 1)};
    return fit_quad_v(v, off);
}

// getTrace (surfd.cu:369-377).  makePoint builds this box from the
// interpolated scale without a bounds check (surfd.cu:1010-1020), so near a
// border a corner can leave [0, W] x [0, H]; the reference then reads the
// flat pitched buffer at that index (column -1 = the previous row's zero
// pad).  Same flat read here; indices outside the frame's buffer read 0.
__device__ __forceinline__ uint32_t flat_at(const uint32_t* __restrict__ I, int idx, int len)
{
    return (idx >= 0 && idx < len) ? I[idx] : 0u;
}
__device__ __forceinline__ uint32_t box_flat(const uint32_t* __restrict__ I, int ip, int len, int x1, int y1,
                                             int x2, int y2)
{
    const int yp1 = (y1 + 1) * ip;
    const int yp2 = y2 * ip;
    return flat_at(I, yp1 + x1 + 1, len) + flat_at(I, yp2 + x2, len) - flat_at(I, yp2 + x1 + 1, len) -
           flat_at(I, yp1 + x2, len);
}
__device__ __forceinline__ int32_t trace_sign(const uint32_t* __restrict__ I, int ip, int len, const int* v)
{
    const int32_t lxx = (int32_t)(box_flat(I, ip, len, v[5] + v[2], v[1] + v[3], v[6] - v[2], v[1] - v[3])
                                  - 3u * box_flat(I, ip, len, v[0] + v[2], v[1] + v[3], v[0] - v[2], v[1] - v[3]));
    const int32_t lyy = (int32_t)(box_flat(I, ip, len, v[0] + v[3], v[7] + v[2], v[0] - v[3], v[8] - v[2])
                                  - 3u * box_flat(I, ip, len, v[0] + v[3], v[1] + v[2], v[0] - v[3], v[1] - v[2]));
    return ((int32_t)((uint32_t)lxx + (uint32_t)lyy) > 0) ? 1 : -1;
}

// Sub-pixel interpolation + acceptance + makePoint (surfd.cu:794-831,
// 942-1022) for one NMS survivor.
// cube: the scan's record of the 19 responses around (s, r, c) (nullptr:
// read them from the planes)
// stash: leave getTrace to k_describe_u2 (trace_in_describe): laplace holds
// its box centre x0 | y0 << 16 (int16 each) and ori the lobe `temp`, which
// the describe kernel replaces by the sign and 0
__device__ bool nms_fit_point(const uint32_t* __restrict__ I, const OctView& V, const FrameParams& P,
                              const OctaveParams& q, int o, int s, int r, int c, const float4* cube,
                              surfhip_point& pt, bool stash)
{
    const int sw = q.sw, sh = q.sh;
    float off[3] = {0.f, 0.f, 0.f};
    float strength = 0.f;
    int newr = r, newc = c;
    for (int mv = 0; mv < 5; mv++) {
        r = newr; c = newc;
        if (mv == 0 && cube) {
            float v[20];
#pragma unroll
            for (int k = 0; k < 5; k++) {
                const float4 t = cube[k];
                v[4 * k] = t.x; v[4 * k + 1] = t.y; v[4 * k + 2] = t.z; v[4 * k + 3] = t.w;
            }
            strength = fit_quad_v(v, off);
        } else {
            strength = fit_quad(V, off, s, r, c);
        }
        const int bs = q.borders[s];
        if (off[1] > 0.6f && r < sh - bs) newr++;
        if (off[1] < -0.6f && r > bs) newr--;
        if (off[2] > 0.6f && c < sw - bs) newc++;
        if (off[2] < -0.6f && c > bs) newc--;
        if (newr == r && newc == c) break;
    }
    if (__builtin_isnan(off[0]) || __builtin_isnan(off[1]) || __builtin_isnan(off[2]) ||
        fabsf(off[0]) > 1.5f || fabsf(off[1]) > 1.5f || fabsf(off[2]) > 1.5f || strength < P.thresh)
        return false;

    const int octave = q.octave;
    const float t2 = (((float)s + off[0]) * 2.f) * (float)octave;
    const float ns = ((float)(P.init_lobe + (octave - 1) * P.max_scale) + t2) / 3.f;
    const float ny = (float)octave * ((float)r + off[1]);
    const float nx = (float)octave * ((float)c + off[2]);
    const float temp_delta = (float)P.sampling * P.divisor;
    pt.x = nx * temp_delta;
    pt.y = ny * temp_delta;
    pt.scale = (1.2f * ns) * P.divisor;
    pt.o = o;
    pt.strength = strength;
    pt.ori = 0.f;
    pt.score = 0.f;
    pt.match = -1;
    pt.match_x = 0.f;
    pt.match_y = 0.f;
    pt.ambiguity = 0.f;
    int v[9];
    const int temp = f2i_rz(fmaf(3.f, ns, 0.5f));
    v[0] = f2i_rz(fmaf(nx, (float)P.sampling, 0.5f));
    v[1] = f2i_rz(fmaf(ny, (float)P.sampling, 0.5f));
    v[2] = temp / 2;
    v[3] = v[2] + v[2];
    v[4] = v[2] + v[3];
    v[5] = v[0] + temp;
    v[6] = v[0] - temp;
    v[7] = v[1] + temp;
    v[8] = v[1] - temp;
    if (stash) {
        pt.laplace = (int)(((uint32_t)v[0] & 0xffffu) | ((uint32_t)v[1] << 16));
        pt.ori = __int_as_float(temp);
    } else {
        pt.laplace = trace_sign(I, P.ip, P.iH * P.ip, v);
    }
    return true;
}

__device__ __forceinline__ OctView make_view(const float* F, const OctaveParams& q, int o)
{
    OctView V;
    V.F = F;
    V.cur = (int)q.ooff;
    V.sp = q.sp;
    V.osize = q.osize;
    V.half = o > 0 ? 1 : 0;
    V.hb = (int)q.hbase[0];
    V.dhb = (int)(q.hbase[1] - q.hbase[0]);
    V.hr = q.hrow[0];
    V.dhr = q.hrow[1] - q.hrow[0];
    V.hc = q.hcol[0];
    V.dhc = q.hcol[1] - q.hcol[0];
    return V;
}

#ifndef SURF_NMS_GLOBAL_ROW3
#define SURF_NMS_GLOBAL_ROW3 0        // (A/B) the neighbour rows of three by global instead of buffer loads
#endif
// Wave-aggregated append: one atomic per wave for all its `ok` lanes.
__device__ __forceinline__ int wave_append(bool ok, int* counter)
{
    const unsigned long long m = __ballot(ok);
    if (m == 0ull) return -1;
    const int leader = __builtin_ctzll(m);
    int base = 0;
    if ((int)lane_id() == leader) base = atomicAdd(counter, (int)__popcll(m));
    base = __shfl(base, leader, 64);
    return ok ? base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u))
              : -1;
}

// Pass 1: the 3x3x3 test for every 2x2x2 block of every octave and both NMS
// levels.  Streams the response planes once; survivors (~1 % of blocks) are
// appended to the frame's scan list with their canonical key (octave, level,
// block row, block col) and argmax (s, r, c).
// One workgroup = 4 waves x (64 block columns x kScanRows/4 block rows) of
// one (frame, octave, level), a wave's rows in passes of 4 whose loads are
// issued one pass ahead; XCD x takes frames x, x + 8, ...
// HK: plane k of this item is a halfImage view (octave > 0, level 1): its
// column pairs are two loads; every other pair is one 8-byte load
template <bool CUBE, bool HK>
__device__ __forceinline__ void nms_scan_item(const float* __restrict__ resp, const FrameParams& P,
                                              const OctaveParams* __restrict__ oct, const LaunchPlan& plan,
                                              uint32_t* __restrict__ scan_key, uint32_t* __restrict__ scan_src,
                                              float* __restrict__ scan_cube,
                                              int* __restrict__ item_count, int nitems_frame, int f, int gb, int wv,
                                              float* sbest, uint32_t* sinfo, float* sblk)
{
    constexpr int NU = 4;                    // block rows per lane per pass
    constexpr int NIT = kScanRows / 4 / NU;  // passes: the next pass's loads are issued first
    const int o = octave_of(plan.nms_start, P.noct, gb);
    const OctaveParams& q = oct[o];
    const int nbx = plan.nms_nbx[o], nby = plan.nms_nby[o];
    int lb = gb - plan.nms_start[o];
    const int z = lb / (nbx * nby);
    lb -= z * nbx * nby;
    const int x = (lb % nbx) * 64 + (int)lane_id();
    const int ybase = (lb / nbx) * kScanRows + wv;     // this wave: rows ybase + 4 u, u < 4 NIT
    const OctView V = make_view(resp + (size_t)f * P.resp_stride, q, o);
    const rsrc_t RF = make_rsrc(resp + (size_t)f * P.resp_stride, (long long)P.resp_stride * 4);
    const int k = 2 * z + 1, mb = q.mb[z];
    const int j = mb + x * 2;
    const int bx0 = (lb % nbx) * 64;
    // survivors go to this wave item's own region (no atomics): kItemCap
    // entries at item * kItemCap, the count in item_count[item]
    const size_t item = ((size_t)f * nitems_frame + gb) * 4 + wv;
    uint32_t* rkey = scan_key + item * kItemCap;
    uint32_t* rsrc_ = scan_src + item * kItemCap;
    float* rcube = scan_cube + item * kCubeCap * kCubeF;
    int nsurv = 0;
    // ---- a pass's 2x2x2 block loads, all issued before any use
    float v[2][NU][8];
    bool in[2][NU];
    auto load = [&](int it, float (&vv)[NU][8], bool (&inn)[NU]) {
#pragma unroll
        for (int u = 0; u < NU; u++) {
            const int y = ybase + 4 * (it * NU + u), i = mb + y * 2;
            inn[u] = x < q.nms_gx && y < q.nms_gy && i < q.sh - mb && j < q.sw - mb;
            const int ii = inn[u] ? i : mb, jj = inn[u] ? j : mb;
            if constexpr (HK) {
                V.pair(k, ii, jj, vv[u][0], vv[u][1]);
                V.pair(k, ii + 1, jj, vv[u][2], vv[u][3]);
            } else {
                V.pair_full(k, ii, jj, vv[u][0], vv[u][1]);
                V.pair_full(k, ii + 1, jj, vv[u][2], vv[u][3]);
            }
            V.pair_full(k + 1, ii, jj, vv[u][4], vv[u][5]);
            V.pair_full(k + 1, ii + 1, jj, vv[u][6], vv[u][7]);
        }
    };
    load(0, v[0], in[0]);
    static_for<NIT>([&](auto itc) {
        constexpr int it = decltype(itc)::value;
        if constexpr (it + 1 < NIT) load(it + 1, v[(it + 1) & 1], in[(it + 1) & 1]);
        const float (&vc)[NU][8] = v[it & 1];
        const bool (&ic)[NU] = in[it & 1];
        const int y0 = ybase + 4 * it * NU;
        // ---- argmax over the 2x2x2 block in the reference's order (k: w,x,y,z;
        // k+1: w,x,y,z), strict '>', threshold and top-scale rejection
        // (surfd.cu:678-756)
        bool cnd[NU];
        float bst[NU];
        int cs[NU];
#pragma unroll
        for (int u = 0; u < NU; u++) {
            int cas = 0;
            float best = vc[u][0];
#pragma unroll
            for (int t = 1; t < 8; t++)
                if (vc[u][t] > best) { best = vc[u][t]; cas = t; }
            cnd[u] = ic[u] && !(best < P.thresh * 0.8f || (k + 1 == P.max_scale - 1 && cas > 3));
#ifdef SURF_DIAG_NMS_NOCAND
            if (best != -1.2345f) cnd[u] = false;
#endif
#ifndef SURF_NMS_NOPRE
            // 4 of the 19 neighbours, (s / si, r / rp, cn), are the adjacent
            // block column of lane -+ 1 (the same block row): a candidate below
            // any of them cannot survive, so it is dropped before the gathers
            // (same result; a lane whose neighbour block lies outside the grid
            // or the wave keeps its candidate for the full test)
            const float ninf = -__builtin_inff();
            const float lmax = ic[u] ? fmaxf(fmaxf(vc[u][0], vc[u][2]), fmaxf(vc[u][4], vc[u][6])) : ninf;
            const float rmax = ic[u] ? fmaxf(fmaxf(vc[u][1], vc[u][3]), fmaxf(vc[u][5], vc[u][7])) : ninf;
            // lane - 1's right column (wave_shr:1) / lane + 1's left column (wave_shl:1)
            const float fromL = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(ninf), __float_as_int(rmax),
                                                                           0x138, 0xf, 0xf, false));
            const float fromR = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(ninf), __float_as_int(lmax),
                                                                           0x130, 0xf, 0xf, false));
            cnd[u] = cnd[u] && !(best < ((cas & 1) ? fromR : fromL));
#endif
            bst[u] = best;
            cs[u] = cas;
        }
        // ---- compact the candidates of the pass's NU rows into dense lanes
        // (LDS), so the 19-neighbour test costs 19 loads per 64 candidates
        unsigned long long m[NU];
        int ncand = 0;
#pragma unroll
        for (int u = 0; u < NU; u++) {
            m[u] = __ballot(cnd[u]);
            if (cnd[u]) {
                const int slot = ncand + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m[u] >> 32),
                                                                       __builtin_amdgcn_mbcnt_lo((unsigned)m[u], 0u));
                sbest[slot] = bst[u];
                sinfo[slot] = ((uint32_t)u << 9) | ((uint32_t)cs[u] << 6) | lane_id();
                // the block's 8 values for the fit record (first 64 candidates)
                if (CUBE && slot < 64) {
                    float4* bd = reinterpret_cast<float4*>(sblk + 8 * slot);
                    bd[0] = make_float4(vc[u][0], vc[u][1], vc[u][2], vc[u][3]);
                    bd[1] = make_float4(vc[u][4], vc[u][5], vc[u][6], vc[u][7]);
                }
            }
            ncand += (int)__popcll(m[u]);
        }
        if (ncand == 0) return;
        wave_sync();
        for (int c0 = 0; c0 < ncand; c0 += 64) {
            const int ci = c0 + (int)lane_id();
            bool ok = false;
            int s = 0, r = 0, c = 0, xx = 0, y = 0, ds = 1, dr = 1, dc = 1;
            int u = 0, cas = 0;
            float best = 0.f, nb[19];
            if (ci < ncand) {
                best = sbest[ci];
                const uint32_t info = sinfo[ci];
                u = (int)(info >> 9); cas = (int)((info >> 6) & 7u);
                xx = bx0 + (int)(info & 63u);
                y = y0 + 4 * u;
                const int i = mb + y * 2, jx = mb + xx * 2;
                s = k + (cas >> 2); r = i + ((cas >> 1) & 1); c = jx + (cas & 1);
                ds = (cas >> 2) ? 1 : -1; dr = ((cas >> 1) & 1) ? 1 : -1; dc = (cas & 1) ? 1 : -1;
                const int so = s + ds, si = s - ds;
                const int rn = r + dr, rp = r - dr, cn = c + dc;
                // the 19 neighbours outside the block, ties survive (surfd.cu:757-792),
                // in six rounds, each only for the candidates the previous
                // ones left: plane s's row rn, its column cn, plane si, then
                // plane so's rows r, rp, rn.  Gathers for every candidate cost
                // half the scan (0.87 ms with all 19 up front, 0.42 without
                // any); in rounds with 12-byte row loads it takes 0.69.
#ifdef SURF_DIAG_NMS_NONB
#define NBV(pl, rr, cc) (best + (float)((pl) + (rr) + (cc)))
#else
#define NBV(pl, rr, cc) V(pl, rr, cc)
#endif
                ok = true;
                // one round of the test: its loads, then its compares (nb keeps
                // the values for the fit record)
                auto test = [&](int at, float v) {
                    nb[at] = v;
                    ok = ok & !(best < v);          // '&': no branch between the loads and a compare
                };
                // (pl, rr, c - 1 .. c + 1): one 12-byte load where plane pl is
                // not a halfImage view
                auto row3 = [&](int at, int pl, int rr) {
                    float a0, a1, a2;
#ifdef SURF_DIAG_NMS_NONB
                    a0 = NBV(pl, rr, c - 1); a1 = NBV(pl, rr, c); a2 = NBV(pl, rr, c + 1);
#else
                    if (HK && pl < 2) {
                        a0 = V(pl, rr, c - 1); a1 = V(pl, rr, c); a2 = V(pl, rr, c + 1);
                    } else {
#if SURF_NMS_GLOBAL_ROW3
                        // (a global 12-byte load: inside the plane -- the block
                        // border keeps r +- 1, c +- 1 in the sample grid)
                        typedef float v3f32a4 __attribute__((ext_vector_type(3), aligned(4)));
                        const v3f32a4 t3 = *reinterpret_cast<const v3f32a4*>(V.F + V.cur + pl * V.osize + rr * V.sp + c - 1);
                        a0 = t3.x; a1 = t3.y; a2 = t3.z;
#else
                        typedef uint32_t v3u32 __attribute__((ext_vector_type(3)));
                        const v3u32 t3 = __builtin_amdgcn_raw_buffer_load_b96(
                            RF, (V.cur + pl * V.osize + rr * V.sp + c - 1) * 4, 0, 0);
                        a0 = __uint_as_float(t3.x); a1 = __uint_as_float(t3.y); a2 = __uint_as_float(t3.z);
#endif
                    }
#endif
                    test(at, a0); test(at + 1, a1); test(at + 2, a2);
                };
                row3(9, s, rn);
                if (ok) { test(12, NBV(s, r, cn)); test(13, NBV(s, rp, cn)); }
                if (ok) { row3(14, si, rn); test(17, NBV(si, rp, cn)); test(18, NBV(si, r, cn)); }
                if (ok) row3(3, so, r);
                if (ok) row3(0, so, rp);
                if (ok) row3(6, so, rn);
#undef NBV
            }
            const unsigned long long mo = __ballot(ok);
            if (ok) {
                const int slot = nsurv + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mo >> 32),
                                                                       __builtin_amdgcn_mbcnt_lo((unsigned)mo, 0u));
                // (octave 3 bits, level 2, block row 13, block column 14): the canonical order
                rkey[slot] = ((uint32_t)o << 29) | ((uint32_t)z << 27) | ((uint32_t)y << 14) | (uint32_t)xx;
                rsrc_[slot] = ((uint32_t)s << 28) | ((uint32_t)r << 14) | (uint32_t)c;
                if (CUBE && slot < kCubeCap) {
                    // the 19 values fitQuadrat's first pass reads (fit_quad),
                    // from the test's registers: k_nms_fit then gathers
                    // nothing for a survivor that does not move; plus the six
                    // block values it needs (the block's opposite corner is
                    // not read), block index cas ^ {col, row, scale} bits, from
                    // the block the candidate's lane staged in LDS at
                    // compaction (a memory reload cost the scan a round trip,
                    // cross-lane reads kept the block registers live: 76 VGPRs)
                    // (a candidate past the first 64 of its pass reloads them:
                    // the fit reads a record for every survivor slot < kCubeCap)
                    float b_r_cm, b_rp_c, b_rp_cm, i_r_c, i_r_cm, i_rp_c;
                    if (ci < 64) {
                        const float* bs = sblk + 8 * ci;
                        b_r_cm = bs[cas ^ 1]; b_rp_c = bs[cas ^ 2]; b_rp_cm = bs[cas ^ 3];
                        i_r_c = bs[cas ^ 4]; i_r_cm = bs[cas ^ 5]; i_rp_c = bs[cas ^ 6];
                    } else {
                        const int si = s - ds, rp = r - dr;
                        b_r_cm = V(s, r, c - dc); b_rp_c = V(s, rp, c); b_rp_cm = V(s, rp, c - dc);
                        i_r_c = V(si, r, c); i_r_cm = V(si, r, c - dc); i_rp_c = V(si, rp, c);
                    }
                    // V(s + a, r + b, c + e) for the positions fit_quad reads
                    // (selects, not indexing: nb stays in registers)
                    auto pick = [](int e, float m, float z, float p) -> float { return e < 0 ? m : (e == 0 ? z : p); };
                    auto so_at = [&](int b, int e) -> float {
                        return b == 0 ? pick(e, nb[3], nb[4], nb[5])
                                      : (b == dr ? pick(e, nb[6], nb[7], nb[8]) : pick(e, nb[0], nb[1], nb[2]));
                    };
                    auto s_at = [&](int b, int e) -> float {
                        if (b == 0) return e == 0 ? best : (e == dc ? nb[12] : b_r_cm);
                        if (b == dr) return pick(e, nb[9], nb[10], nb[11]);
                        return e == 0 ? b_rp_c : (e == dc ? nb[13] : b_rp_cm);
                    };
                    auto si_at = [&](int b, int e) -> float {       // no corner is read
                        if (b == 0) return e == 0 ? i_r_c : (e == dc ? nb[18] : i_r_cm);
                        if (b == dr) return pick(e, nb[14], nb[15], nb[16]);
                        return i_rp_c;
                    };
                    auto at = [&](int a, int b, int e) -> float {
                        return a == 0 ? s_at(b, e) : (a == ds ? so_at(b, e) : si_at(b, e));
                    };
                    float4* dst = reinterpret_cast<float4*>(rcube + (size_t)slot * kCubeF);
                    dst[0] = make_float4(best, at(1, 0, 0), at(-1, 0, 0), at(0, 1, 0));
                    dst[1] = make_float4(at(0, -1, 0), at(0, 0, 1), at(0, 0, -1), at(1, 1, 0));
                    dst[2] = make_float4(at(1, -1, 0), at(-1, 1, 0), at(-1, -1, 0), at(1, 0, 1));
                    dst[3] = make_float4(at(1, 0, -1), at(-1, 0, 1), at(-1, 0, -1), at(0, 1, 1));
                    dst[4] = make_float4(at(0, 1, -1), at(0, -1, 1), at(0, -1, -1), 0.f);
                }
            }
            nsurv += (int)__popcll(mo);
        }
        wave_sync();                          // sbest / sinfo are rewritten by the next pass
    });
    // every item writes its count, zero included (no per-batch memset)
    if (lane_id() == 0u) item_count[item] = nsurv;
}

// CUBE: write the survivors' fit records (k_nms_fit's first pass then reads
// no planes); without it the scan keeps 38 instead of 76 VGPRs, which single
// frames (config #2: a few hundred survivors) prefer
template <bool CUBE>
__global__ __launch_bounds__(256) void k_nms_scan(const float* __restrict__ resp, FrameParams P,
                                                  const OctaveParams* __restrict__ oct, LaunchPlan plan,
                                                  uint32_t* __restrict__ scan_key, uint32_t* __restrict__ scan_src,
                                                  float* __restrict__ scan_cube, int* __restrict__ item_count,
                                                  int nframes, int* __restrict__ cand_count, int* __restrict__ status)
{
    __shared__ float sbest[4][64 * 4];                // one pass's candidates per wave
    __shared__ __attribute__((aligned(16))) float sblk[4][64 * 8];   // blocks of its first 64 (CUBE)
    __shared__ uint32_t sinfo[4][64 * 4];
    int f, gb;
    if (!xcd_frame_block(plan.nms_start[kMaxOct], nframes, f, gb)) return;
    // the batch's counters the fit and sort use after this kernel: the
    // frame's accepted-candidate count and the truncation flag (no memsets)
    if (gb == 0 && threadIdx.x == 0) {
        cand_count[f] = 0;
        if (f == 0) *status = 0;
    }
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // plane k (= 2 z + 1) is a halfImage view for octaves > 0 at level z = 0
    const int o = octave_of(plan.nms_start, P.noct, gb);
    const int z = (gb - plan.nms_start[o]) / (plan.nms_nbx[o] * plan.nms_nby[o]);
    if (o > 0 && z == 0)
        nms_scan_item<CUBE, true>(resp, P, oct, plan, scan_key, scan_src, scan_cube, item_count,
                                  plan.nms_start[kMaxOct], f, gb, wv, sbest[wv], sinfo[wv], sblk[wv]);
    else
        nms_scan_item<CUBE, false>(resp, P, oct, plan, scan_key, scan_src, scan_cube, item_count,
                                   plan.nms_start[kMaxOct], f, gb, wv, sbest[wv], sinfo[wv], sblk[wv]);
}

// Exclusive prefix of n ints (n up to ~2M): each workgroup scans 2048
// elements (block_excl_scan) and records its total, one workgroup scans the
// totals, then the block offsets are added.  out[n] = total.
constexpr int kScanChunk = 2048;

__global__ __launch_bounds__(256) void k_scan_local(const int* __restrict__ in, int n, int* __restrict__ out,
                                                    int* __restrict__ bsum)
{
    __shared__ uint32_t lds4[4];
    const int b0 = blockIdx.x * kScanChunk + threadIdx.x * 8;
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = (b0 + k < n) ? (uint32_t)in[b0 + k] : 0u;
    const uint32_t last = v[7];
    block_excl_scan<8>(v, lds4);
#pragma unroll
    for (int k = 0; k < 8; k++)
        if (b0 + k < n) out[b0 + k] = (int)v[k];
    if (threadIdx.x == 255) {
        // one chunk (n <= kScanChunk: a frame or two's NMS items): the total
        // goes straight to out[n] and the other two kernels are not launched
        if (gridDim.x == 1) out[n] = (int)(v[7] + last);
        else bsum[blockIdx.x] = (int)(v[7] + last);
    }
}

__global__ __launch_bounds__(1024) void k_scan_top(int* __restrict__ bsum, int nb, int* __restrict__ out, int n)
{
    __shared__ int part[16];
    const int per = (nb + 1023) / 1024;
    const int b = threadIdx.x * per;
    int sum = 0;
    for (int i = 0; i < per; i++) if (b + i < nb) sum += bsum[b + i];
    // exclusive scan of the 1,024 partial sums: DPP wave scans and the 16
    // wave totals (was one thread walking all 1,024)
    const uint32_t inc = wave_incl_scan((uint32_t)sum);
    const int wv = (int)(threadIdx.x >> 6);
    if (lane_id() == 63) part[wv] = (int)inc;
    __syncthreads();
    uint32_t wbase = 0u, total = 0u;
    for (int t = 0; t < 16; t++) {
        const uint32_t v = (uint32_t)part[t];
        wbase += t < wv ? v : 0u;
        total += v;
    }
    if (threadIdx.x == 0) out[n] = (int)total;
    int run = (int)(wbase + inc) - sum;
    for (int i = 0; i < per; i++)
        if (b + i < nb) { const int v = bsum[b + i]; bsum[b + i] = run; run += v; }
}

__global__ __launch_bounds__(256) void k_scan_add(int* __restrict__ out, int n, const int* __restrict__ bsum)
{
    const int add = bsum[blockIdx.x];
    const int b0 = blockIdx.x * kScanChunk;
    for (int i = threadIdx.x; i < kScanChunk && b0 + i < n; i += 256) out[b0 + i] += add;
}

static void launch_excl_scan(const int* in, int n, int* out, int* bsum, hipStream_t s)
{
    const int nb = (n + kScanChunk - 1) / kScanChunk;
    k_scan_local<<<nb, 256, 0, s>>>(in, n, out, bsum);
    if (nb == 1) return;
    k_scan_top<<<1, 1024, 0, s>>>(bsum, nb, out, n);
    k_scan_add<<<nb, 256, 0, s>>>(out, n, bsum);
}

// k_nms_fit's grid: 5 waves per SIMD fit (90 VGPRs) = 1,280 workgroups of 4
// waves; SURFHIP_FIT_GRID overrides (A/B)
static int fit_grid()
{
    static const int g = getenv("SURFHIP_FIT_GRID") ? std::max(64, atoi(getenv("SURFHIP_FIT_GRID"))) : 1280;
    return g;
}

// Pass 2: interpolation + makePoint, one lane per survivor of the whole batch
// (grid-stride over the prefix of the scan items' survivor counts), so no
// lane idles on the ~99 % of blocks that fail the 3x3x3 test and no
// workgroup is launched for empty space.
__global__ __launch_bounds__(256) void k_nms_fit(const int32_t* __restrict__ ii, const float* __restrict__ resp,
                                                 FrameParams P, const OctaveParams* __restrict__ oct,
                                                 const uint32_t* __restrict__ scan_key,
                                                 const uint32_t* __restrict__ scan_src,
                                                 const float* __restrict__ scan_cube,
                                                 const int* __restrict__ soff, int nitems, int items_per_frame,
                                                 surfhip_point* __restrict__ cand, uint32_t* __restrict__ keys,
                                                 int* __restrict__ cand_count, int cap, int stash)
{
    const int total = soff[nitems];
    const int stride = (int)gridDim.x * 256;
    for (int base = blockIdx.x * 256 + (threadIdx.x & ~63); base < total; base += stride) {
        const int t = base + (int)lane_id();
        const bool act = t < total;
        int f = 0;
        surfhip_point pt;
        bool ok = false;
        uint32_t key = 0;
        // the scan item holding each lane's survivor t = base + lane: the
        // wave finds base's item by a 64-way search (one coalesced load of
        // 64 probes per level: ~3-4 levels instead of a lane's ~19 dependent
        // loads), then lane t counts the item starts after it that are <= t
        // among the next 64 (ascending: a 6-step search over the lanes'
        // values); a lane past those 64 items searches on its own
        int wlo = 0;
        {
            int hi = nitems;                                 // soff[wlo] <= base < soff[hi]
            while (hi - wlo > 1) {
                const int sw = (hi - wlo + 63) >> 6;
                const int pr = wlo + ((int)lane_id() + 1) * sw;
                const bool le = pr < hi && soff[pr] <= base;
                const unsigned long long m = __ballot(le);
                const int k = m ? 64 - __builtin_clzll(m) : 0;
                wlo += k * sw;
                hi = min(wlo + sw, hi);
            }
        }
        const int wi = wlo + 1 + (int)lane_id();
        const int wst = wi <= nitems ? soff[wi] : 0x7fffffff; // item starts after wlo, ascending
        int cnt = 0;
#pragma unroll
        for (int sft = 32; sft >= 1; sft >>= 1) {
            const int v = __shfl(wst, cnt + sft - 1, 64);
            if (v <= t) cnt += sft;
        }
        if (cnt == 63 && __shfl(wst, 63, 64) <= t) cnt = 64;      // (all 64 starts <= t)
        if (act) {
            int lo = wlo + cnt;                          // scan item holding survivor t
            if (cnt == 64) {
                int hi = nitems;
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (soff[mid] <= t) lo = mid; else hi = mid;
                }
            }
            f = lo / items_per_frame;
            const int idx = t - soff[lo];                // survivor index within its scan item
            const size_t src_i = (size_t)lo * kItemCap + idx;
            key = scan_key[src_i];
            const uint32_t src = scan_src[src_i];
            const int o = (int)(key >> 29);
            const OctaveParams& q = oct[o];
            const OctView V = make_view(resp + (size_t)f * P.resp_stride, q, o);
            const uint32_t* I = reinterpret_cast<const uint32_t*>(ii) + (size_t)f * P.ii_stride;
            const float4* cube = idx < kCubeCap && scan_cube
                ? reinterpret_cast<const float4*>(scan_cube + ((size_t)lo * kCubeCap + idx) * kCubeF) : nullptr;
#ifndef SURF_DIAG_NOFIT
            ok = nms_fit_point(I, V, P, q, o, (int)(src >> 28), (int)((src >> 14) & 0x3fffu), (int)(src & 0x3fffu),
                               cube, pt, stash != 0);
#else
            ok = (src & 1u) && I != nullptr && V.F != nullptr && cube != nullptr;
#endif
        }
        // Survivor t of frame f goes to slot t - (f's first survivor): the
        // slots are the survivors' scan order, so which candidates a frame
        // with more than `cap` survivors keeps is deterministic (the first
        // cap survivors; k_sort then orders them canonically).  A rejected
        // survivor leaves an invalid key, sorted last.
        if (act) {
            const int slot = t - soff[f * items_per_frame];
            if (slot < cap) {
                if (ok) cand[(size_t)f * cap + slot] = pt;
                keys[(size_t)f * cap + slot] = ok ? key : kNoKey;
            }
        }
        // accepted candidates per frame (a wave spans at most a few frames);
        // k_sort compares it with the ones inside the cap to flag truncation
        bool pending = ok;
        while (__ballot(pending)) {
            const int leader = __builtin_ctzll(__ballot(pending));
            const int ff = __shfl(f, leader, 64);
            const bool mine = pending && f == ff;
            const unsigned long long m = __ballot(mine);
            if ((int)lane_id() == leader) atomicAdd(&cand_count[ff], __popcll(m));
            if (mine) pending = false;
        }
    }
}

hipError_t launch_nms(const int32_t* ii, const float* resp, int nframes, const FrameParams& P,
                      const OctaveParams* d_oct, const LaunchPlan& plan, uint32_t* scan_key, uint32_t* scan_src,
                      float* scan_cube, int* item_count, int* item_off, surfhip_point* cand, uint32_t* keys,
                      int* cand_count, int cap, int* status, hipStream_t s, bool stash_trace)
{
    const int per = plan.nms_start[kMaxOct];
    if (per == 0) {
        // (no NMS level: nothing to scan; the counters the sort reads are 0)
        hipError_t e = hipMemsetAsync(cand_count, 0, sizeof(int) * (size_t)nframes, s);
        if (e == hipSuccess) e = hipMemsetAsync(status, 0, sizeof(int), s);
        return e;
    }
    // the scan's fit records for every batch size (round 5: one 1080p frame's
    // NMS 0.038 -> 0.034 ms with them; round 2's cross-lane variant had made
    // single frames slower)
    static const char* ce = getenv("SURFHIP_FIT_CUBE");                  // A/B: 0 off, 1 on
    const bool cube = ce ? atoi(ce) != 0 : true;
    if (!cube) scan_cube = nullptr;
    auto* scan = cube ? &k_nms_scan<true> : &k_nms_scan<false>;
    scan<<<dim3(frame_grid(nframes) * per), 256, 0, s>>>(resp, P, d_oct, plan, scan_key, scan_src, scan_cube,
                                                                item_count, nframes, cand_count, status);
    const int nitems = nframes * per * 4;
    launch_excl_scan(item_count, nitems, item_off, item_off + nitems + 1, s);
    k_nms_fit<<<fit_grid(), 256, 0, s>>>(ii, resp, P, d_oct, scan_key, scan_src, scan_cube, item_off, nitems, per * 4,
                                         cand, keys, cand_count, cap, stash_trace ? 1 : 0);
    return hipGetLastError();
}

// ======================================================================
// Canonical order + max_pts cap.  The reference emits in atomicInc order
// and can write past max_pts (surfd.cu:827-830, no pi<max guard); here each
// frame's candidates are sorted by key (bitonic, in LDS up to kSortCap, in
// a global scratch beyond) and the first max_pts are kept.
// ======================================================================

template <typename PtrT>
__device__ void bitonic_sort(PtrT s, int n)
{
    for (int k = 2; k <= n; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t a = s[i], b = s[ixj];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) { s[i] = b; s[ixj] = a; }
                }
            }
            __syncthreads();
        }
    }
}

// The same network on an LDS array with 1024 threads: pair p of pass (k, j)
// is elements (i, i + j), i = 2p - (p mod j), so every thread works every
// pass, and a wave's 64 pairs (p = 64 w .. 64 w + 63 + 1024 m) cover the
// 128-element blocks [128 (w + 16 m), +128) whenever j <= 64: those passes
// need only a wave-level sync; a block barrier is kept around every pass
// with j >= 128 (63 of the 78 passes of a 4,096-key sort skip it).
__device__ void bitonic_sort_lds(uint64_t* s, int n)
{
    const int npairs = n >> 1;
    for (int k = 2; k <= n; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int p = threadIdx.x; p < npairs; p += 1024) {
                const int i = 2 * p - (p & (j - 1));
                const uint64_t a = s[i], b = s[i + j];
                const bool up = (i & k) == 0;
                if ((a > b) == up) { s[i] = b; s[i + j] = a; }
            }
            const int nj = j > 1 ? j >> 1 : k;          // the next pass's distance
            if (j >= 128 || (nj >= 128 && k < n)) __syncthreads();
            else wave_sync();
        }
    }
    __syncthreads();
}

// The value of lane (lane ^ J) (J = 1 .. 32) of a 64-bit element, by DPP /
// permlane swaps (no LDS round trip).
template <int J>
__device__ __forceinline__ uint32_t xor_lane32(uint32_t v, int lane)
{
    if constexpr (J == 1) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
    } else if constexpr (J == 2) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
    } else if constexpr (J == 4 || J == 8) {
        const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 + J, 0xf, 0xf, false);   // lane + J
        const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 + J, 0xf, 0xf, false);   // lane - J
        return (lane & J) ? dn : up;
    } else {
        auto r = J == 16 ? __builtin_amdgcn_permlane16_swap(v, v, false, false)
                         : __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & J) ? r[0] : r[1];
    }
}
template <int J>
__device__ __forceinline__ uint64_t xor_lane64(uint64_t v, int lane)
{
    return ((uint64_t)xor_lane32<J>((uint32_t)(v >> 32), lane) << 32) | xor_lane32<J>((uint32_t)v, lane);
}
// One compare-exchange pass (k, J <= 32) of a 128-element block held two per
// lane (positions lane and lane + 64 of the block starting at `base`).
template <int J>
__device__ __forceinline__ void bitonic_reg_pass(uint64_t& e0, uint64_t& e1, int base, int k, int lane)
{
    const uint64_t p0 = xor_lane64<J>(e0, lane), p1 = xor_lane64<J>(e1, lane);
    const bool lower = (lane & J) == 0;
    const bool up0 = ((base + lane) & k) == 0, up1 = ((base + lane + 64) & k) == 0;
    e0 = (lower == up0) ? (e0 < p0 ? e0 : p0) : (e0 < p0 ? p0 : e0);
    e1 = (lower == up1) ? (e1 < p1 ? e1 : p1) : (e1 < p1 ? p1 : e1);
}
__device__ __forceinline__ void bitonic_reg_tail(uint64_t& e0, uint64_t& e1, int base, int k, int jmax, int lane)
{
    // passes J = jmax .. 1 (jmax <= 32)
    if (jmax >= 32) bitonic_reg_pass<32>(e0, e1, base, k, lane);
    if (jmax >= 16) bitonic_reg_pass<16>(e0, e1, base, k, lane);
    if (jmax >= 8) bitonic_reg_pass<8>(e0, e1, base, k, lane);
    if (jmax >= 4) bitonic_reg_pass<4>(e0, e1, base, k, lane);
    if (jmax >= 2) bitonic_reg_pass<2>(e0, e1, base, k, lane);
    bitonic_reg_pass<1>(e0, e1, base, k, lane);
}

// The same network with every pass of distance <= 64 in registers: a wave
// holds a 128-element block two per lane and runs those passes with DPP /
// permlane swaps; only the passes of distance >= 128 go through LDS (with a
// workgroup barrier each).  n >= 128, blockDim.x == 1024.
__device__ void bitonic_sort_lds_reg(uint64_t* s, int n)
{
    const int lane = (int)lane_id(), wv = (int)(threadIdx.x >> 6);
    const int nblk = n >> 7;
    // k = 2 .. 64: within blocks only
    for (int b = wv; b < nblk; b += 16) {
        const int base = b << 7;
        uint64_t e0 = s[base + lane], e1 = s[base + lane + 64];
        for (int k = 2; k <= 64; k <<= 1) bitonic_reg_tail(e0, e1, base, k, k >> 1, lane);
        s[base + lane] = e0;
        s[base + lane + 64] = e1;
    }
    __syncthreads();
    const int npairs = n >> 1;
    for (int k = 128; k <= n; k <<= 1) {
        for (int j = k >> 1; j >= 128; j >>= 1) {
            for (int p = threadIdx.x; p < npairs; p += 1024) {
                const int i = 2 * p - (p & (j - 1));
                const uint64_t a = s[i], b = s[i + j];
                const bool up = (i & k) == 0;
                if ((a > b) == up) { s[i] = b; s[i + j] = a; }
            }
            __syncthreads();
        }
        for (int b = wv; b < nblk; b += 16) {
            const int base = b << 7;
            uint64_t e0 = s[base + lane], e1 = s[base + lane + 64];
            // distance 64: the lane's own two elements
            const bool up = (base & k) == 0;
            if ((e0 > e1) == up) { const uint64_t t = e0; e0 = e1; e1 = t; }
            bitonic_reg_tail(e0, e1, base, k, 32, lane);
            s[base + lane] = e0;
            s[base + lane + 64] = e1;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(1024) void k_sort(const surfhip_point* __restrict__ cand,
                                               const uint32_t* __restrict__ keys,
                                               uint64_t* __restrict__ gscratch, const int* __restrict__ cand_count,
                                               const int* __restrict__ soff, int items_per_frame, int cap,
                                               surfhip_point* __restrict__ out, int max_pts,
                                               int* __restrict__ out_count, int* __restrict__ order, int* status)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t sk[];
    __shared__ int nvalid;
    const int f = blockIdx.x;
    // slots written by k_nms_fit: the frame's survivors, at most cap
    const int cnt = min(soff[(f + 1) * items_per_frame] - soff[f * items_per_frame], cap);
    int n = 1;
    while (n < cnt) n <<= 1;                  // <= cap (a power of 2)
    const bool in_lds = n <= kSortCap;
    uint64_t* s = in_lds ? sk : gscratch + (size_t)f * cap;
    if (threadIdx.x == 0) nvalid = 0;
    __syncthreads();
    int mine = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t k = (i < cnt) ? keys[(size_t)f * cap + i] : kNoKey;
        mine += k != kNoKey;
        s[i] = ((uint64_t)k << 32) | (uint32_t)i;
    }
    if (mine) atomicAdd(&nvalid, mine);
    __syncthreads();
#ifdef SURF_SORT_LDSONLY
    if (in_lds && blockDim.x == 1024) bitonic_sort_lds(s, n);
#else
    if (in_lds && blockDim.x == 1024 && n >= 128) bitonic_sort_lds_reg(s, n);
    else if (in_lds && blockDim.x == 1024) bitonic_sort_lds(s, n);
#endif
    else bitonic_sort(s, n);
    const int valid = nvalid;
    // accepted candidates beyond the cap were dropped: report it
    if (threadIdx.x == 0 && cand_count[f] > valid) atomicOr(status, 1);
    const int keep = min(valid, max_pts);
    for (int t = threadIdx.x; t < keep; t += blockDim.x)
        out[(size_t)f * max_pts + t] = cand[(size_t)f * cap + (uint32_t)(s[t] & 0xffffffffu)];
    if (threadIdx.x == 0) out_count[f] = keep;
    // Describe schedule (processing order only; descriptors land at their
    // canonical index): keypoints in 16-row bands of the frame, canonical
    // order within a band.  The canonical order sweeps the frame 2 x noctaves
    // times (octave, layer, y); the band order sweeps it once, so the few
    // hundred keypoints an XCD describes at a time share their integral-image
    // rows in that XCD's L2.
    // (SURF_DESC_BAND_SHIFT: log2 of the band height, A/B)
#ifndef SURF_DESC_BAND_SHIFT
#define SURF_DESC_BAND_SHIFT 4
#endif
// A counting sort by band: the order within a band is free (describe
    // writes each descriptor at its canonical index; the order only groups
    // the keypoints an XCD describes at a time), so two passes of LDS atomics
    // replace round 2's second bitonic sort (78 barrier passes for 4,096 keys).
    int* ord = order + (size_t)f * max_pts;
    __threadfence_block();
    __syncthreads();                          // s[] is dead, out[] is written
    constexpr int NBAND = 4096;               // 16-row bands of frames up to 65,536 rows
    uint32_t* bc = reinterpret_cast<uint32_t*>(sk);
    __shared__ uint32_t wsum[32];
    for (int b = threadIdx.x; b < NBAND; b += blockDim.x) bc[b] = 0u;
    __syncthreads();
    auto band_of = [&](int t) -> uint32_t {
        const float y = out[(size_t)f * max_pts + t].y;
        return min((uint32_t)max(y, 0.f) >> SURF_DESC_BAND_SHIFT, (uint32_t)NBAND - 1u);
    };
    for (int t = threadIdx.x; t < keep; t += blockDim.x) atomicAdd(&bc[band_of(t)], 1u);
    __syncthreads();
    {
        constexpr int PER = NBAND / 1024;     // blockDim.x == 1024
        uint32_t v[PER];
#pragma unroll
        for (int k = 0; k < PER; k++) v[k] = bc[PER * threadIdx.x + k];
        block_excl_scan<PER>(v, wsum);
#pragma unroll
        for (int k = 0; k < PER; k++) bc[PER * threadIdx.x + k] = v[k];
    }
    __syncthreads();
    for (int t = threadIdx.x; t < keep; t += blockDim.x) ord[atomicAdd(&bc[band_of(t)], 1u)] = t;
}

// Small batches (nframes <= kRankBatch): the canonical order by ranks,
// spread over many workgroups per frame instead of one bitonic workgroup
// (config #2: one frame's sort ran on one CU of 256).  Valid keys are unique
// (one survivor per 2x2x2 block), so a valid candidate's rank is the number
// of keys below its own -- exactly its position in the bitonic result;
// rejected slots (kNoKey) sort last and are dropped.  Workgroup r of a frame
// ranks candidates [256 r, 256 r + 256) against all of the frame's keys
// (staged in LDS when they fit).  Processing order for describe = canonical.
constexpr int kRankBatch = 8;
constexpr int kRankLds = 16384;
// Rank sort of a frame's candidates (small batches): a valid key's rank
// among the frame's keys is its canonical position (keys are unique).  16
// lanes share a candidate, each counting the smaller keys in every 16th slot
// (lane-interleaved LDS reads), then a 16-lane DPP sum: 16 candidates per
// workgroup.  (One lane per candidate walked all ~3,000 keys of a 1080p
// frame on one wave per SIMD of a dozen CUs: 27-29 us per frame.)
constexpr int kRankT = 16;                      // lanes per candidate
constexpr int kRankMaxWgs = 256;                // workgroups per frame at most
__global__ __launch_bounds__(256) void k_sort_rank(const surfhip_point* __restrict__ cand,
                                                   const uint32_t* __restrict__ keys,
                                                   const int* __restrict__ cand_count,
                                                   const int* __restrict__ soff, int items_per_frame, int cap,
                                                   int wgs_per_frame, surfhip_point* __restrict__ out, int max_pts,
                                                   int* __restrict__ out_count, int* __restrict__ order,
                                                   int* __restrict__ status)
{
    __shared__ __attribute__((aligned(16))) uint32_t sk[kRankLds];
    __shared__ int nvalid;
    constexpr int CPW = 256 / kRankT;           // candidates per workgroup
    const int f = blockIdx.x / wgs_per_frame, r = blockIdx.x - f * wgs_per_frame;
    const int cnt = min(soff[(f + 1) * items_per_frame] - soff[f * items_per_frame], cap);
    const uint32_t* fk = keys + (size_t)f * cap;
    if (r > 0 && r * CPW >= cnt) return;        // nothing to rank here (workgroup 0 writes the count)
    if (threadIdx.x == 0) nvalid = 0;
    __syncthreads();
    const bool lds = cnt <= kRankLds;
    int mine = 0;
    // 8 loads in flight per thread (a loop of single loads waited a memory
    // latency per 256 keys)
    for (int i0 = threadIdx.x; i0 < cnt; i0 += 256 * 8) {
        uint32_t k[8];
#pragma unroll
        for (int u = 0; u < 8; u++) k[u] = (i0 + 256 * u < cnt) ? fk[i0 + 256 * u] : kNoKey;
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (i0 + 256 * u < cnt) {
                if (lds) sk[i0 + 256 * u] = k[u];
                mine += k[u] != kNoKey;
            }
    }
    if (mine) atomicAdd(&nvalid, mine);
    __syncthreads();
    const int valid = nvalid;
    const int keep = min(valid, max_pts);
    if (r == 0 && threadIdx.x == 0) {
        out_count[f] = keep;
        if (cand_count[f] > valid) atomicOr(status, 1);
    }
    const int part = (int)(threadIdx.x & (kRankT - 1));
    // candidate groups r, r + wgs, ...: a dense frame (cnt up to the cap)
    // reuses the keys staged in LDS for several groups instead of restaging
    // them in cnt / 16 workgroups (16x the key loads)
    for (int g = r; g * CPW < cnt; g += wgs_per_frame) {
        const int i = g * CPW + (int)(threadIdx.x / kRankT);
        const uint32_t ki = (i < cnt) ? (lds ? sk[i] : fk[i]) : kNoKey;
        int rank = 0;
        if (ki != kNoKey) {
            if (lds) {
                int j = part;
                for (; j + 7 * kRankT < cnt; j += 8 * kRankT) {
                    uint32_t q[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) q[u] = sk[j + u * kRankT];
#pragma unroll
                    for (int u = 0; u < 8; u++) rank += q[u] < ki;
                }
                for (; j < cnt; j += kRankT) rank += sk[j] < ki;
            } else {
                for (int j = part; j < cnt; j += kRankT) rank += fk[j] < ki;
            }
        }
        // the 16 partial counts of a candidate: DPP row shifts (16-lane rows)
        rank += __builtin_amdgcn_update_dpp(0, rank, 0x111, 0xf, 0xf, false);      // row_shr:1
        rank += __builtin_amdgcn_update_dpp(0, rank, 0x112, 0xf, 0xf, false);      // row_shr:2
        rank += __builtin_amdgcn_update_dpp(0, rank, 0x114, 0xf, 0xf, false);      // row_shr:4
        rank += __builtin_amdgcn_update_dpp(0, rank, 0x118, 0xf, 0xf, false);      // row_shr:8
        // lane 15 of each row holds the row's sum
        if (part == kRankT - 1 && ki != kNoKey && rank < keep) {
            out[(size_t)f * max_pts + rank] = cand[(size_t)f * cap + i];
            order[(size_t)f * max_pts + rank] = rank;
        }
    }
}

__global__ __launch_bounds__(1024) void k_offsets(const int* __restrict__ counts, int nframes, int* __restrict__ offsets)
{
    __shared__ int part[16];
    const int per = (nframes + 1023) / 1024;
    const int b = threadIdx.x * per;
    int sum = 0;
    for (int i = 0; i < per; i++) if (b + i < nframes) sum += counts[b + i];
    // exclusive scan of the 1,024 partial sums: DPP wave scans and the 16
    // wave totals (was one thread walking all 1,024: ~10 us, on config #2's
    // single-frame path too)
    const uint32_t inc = wave_incl_scan((uint32_t)sum);
    const int wv = (int)(threadIdx.x >> 6);
    if (lane_id() == 63) part[wv] = (int)inc;
    __syncthreads();
    uint32_t wbase = 0u, total = 0u;
    for (int t = 0; t < 16; t++) {
        const uint32_t v = (uint32_t)part[t];
        wbase += t < wv ? v : 0u;
        total += v;
    }
    if (threadIdx.x == 0) offsets[nframes] = (int)total;
    int run = (int)(wbase + inc) - sum;
    for (int i = 0; i < per; i++)
        if (b + i < nframes) { offsets[b + i] = run; run += counts[b + i]; }
}

hipError_t launch_sort(const surfhip_point* cand, const uint32_t* keys, uint64_t* gscratch,
                       const int* cand_count, const int* soff, int items_per_frame, int cap, int nframes,
                       surfhip_point* out, int max_pts, int* out_count, int* offsets, int* order, int* status,
                       hipStream_t s)
{
    if (nframes <= kRankBatch && getenv("SURFHIP_SORT_BITONIC") == nullptr) {
        // workgroups per frame: one per 16 candidates up to 256 (~3,000
        // candidates of a 1080p frame: 188), beyond that each takes several
        // groups of 16 with the keys it staged once
        const int per = std::min((cap + 256 / kRankT - 1) / (256 / kRankT), kRankMaxWgs);
        k_sort_rank<<<nframes * per, 256, 0, s>>>(cand, keys, cand_count, soff, items_per_frame, cap, per, out,
                                                  max_pts, out_count, order, status);
    } else {
        hipError_t e = set_max_lds(reinterpret_cast<const void*>(&k_sort), (int)(kSortCap * sizeof(uint64_t)));
        if (e != hipSuccess) return e;
        k_sort<<<nframes, 1024, kSortCap * sizeof(uint64_t), s>>>(cand, keys, gscratch, cand_count, soff,
                                                                  items_per_frame, cap, out, max_pts, out_count,
                                                                  order, status);
    }
    k_offsets<<<1, 1024, 0, s>>>(out_count, nframes, offsets);
    return hipGetLastError();
}

// ======================================================================
// Orientation + descriptor + normalize, one wave (64 lanes) per keypoint,
// 4 keypoints per 256-thread workgroup, grid-strided over all keypoints of
// the batch.  Haar responses are gathered from the integral image (L1/L2);
// descriptor bins accumulate with LDS float atomics (order-free, like the
// reference's global atomics, surfd.cu:1222-1266); the orientation
// histogram is reduced in fixed sample order so `ori` is reproducible.
// ======================================================================

__device__ __forceinline__ int32_t wavelet1(const uint32_t* __restrict__ I, int ip, int x, int y, int size)
{
    return (int32_t)(box(I, ip, x + size, y, x - size, y - size) - box(I, ip, x + size, y + size, x - size, y));
}
__device__ __forceinline__ int32_t wavelet2(const uint32_t* __restrict__ I, int ip, int x, int y, int size)
{
    return (int32_t)(box(I, ip, x + size, y + size, x, y - size) - box(I, ip, x, y + size, x - size, y - size));
}

// dFastAtan2 (surfd.cu:114-126)
__device__ __forceinline__ float fast_atan2(float y, float x)
{
    const float absx = fabsf(x), absy = fabsf(y);
    const float a = fminf(absx, absy) / fmaxf(absx, absy);
    const float s = a * a;
    float r = fmaf(fmaf(fmaf(-0.0464964749f, s, 0.15931422f), s, -0.327622764f), s * a, a);
    r = (absy > absx ? H_PI_F - r : r);
    r = (x < 0 ? (float)(M_PI_D - (double)r) : r);
    r = (y < 0 ? -r : r);
    return r;
}

// Deterministic sin/cos standing in for __sinf/__cosf (surfd.cu:2423-2424);
// identical operation sequence to the oracle's or_sinf/or_cosf.
__device__ __forceinline__ float sincos_poly(float x, int want_cos)
{
    const float q = x * 0.636619772f;
    const float kf = __builtin_rintf(q);
    int k = (int)kf;
    const float r = ((x - kf * 1.5703125f) - kf * 4.837512969970703125e-4f) - kf * 7.54978995489188216e-8f;
    const float z = r * r;
    float ps = -1.9515295891e-4f * z;
    ps = ps + 8.3321608736e-3f;
    ps = ps * z;
    ps = ps - 1.6666654611e-1f;
    ps = ps * z;
    ps = ps * r;
    const float sn = ps + r;
    float pc = 2.443315711809948e-5f * z;
    pc = pc - 1.388731625493765e-3f;
    pc = pc * z;
    pc = pc + 4.166664568298827e-2f;
    pc = pc * z;
    pc = pc * z;
    const float cs = (pc - 0.5f * z) + 1.0f;
    k += want_cos;
    switch (k & 3) {
        case 0: return sn;
        case 1: return cs;
        case 2: return -sn;
        default: return -cs;
    }
}

// x / y as the IEEE quotient, from r = 1 / y (IEEE, once per keypoint): q0 =
// x r, q = q0 + (x - q0 y) r with the remainder exact (fma).  This is the
// correctly rounded x / y whenever the quotient is a normal number (Markstein;
// 0 mismatches in 8.5e8 trials incl. all-ones significands of y); for |x / y|
// below 2^-100 it may differ in the last bits of a value that only ever enters
// rpos + wofs and rpos^2 + cpos^2, where it vanishes.  3 full-rate
// instructions instead of the ~10 of the IEEE division sequence.
__device__ __forceinline__ float div_by(float x, float y, float r)
{
    const float q0 = x * r;
    return __builtin_fmaf(__builtin_fmaf(-q0, y, x), r, q0);
}

// placeInIndex (surfd.cu:1199-1271) into an LDS descriptor.
__device__ __forceinline__ void place(float* d, int wsz, int osz, float mag1, int ori1, float mag2, int ori2,
                                      float rx, float cx)
{
    const int ri = f2i_rz(rx >= 0.f ? rx : rx - 1.f);
    const int ci = f2i_rz(cx >= 0.f ? cx : cx - 1.f);
    const float rfrac = rx - (float)ri;
    const float cfrac = cx - (float)ci;
    const float cfrac1 = 1 - cfrac;
    if (ri >= 0) {
        const float rw1 = mag1 * (1.f - rfrac), rw2 = mag2 * (1.f - rfrac);
        if (ci >= 0) {
            const int o0 = ri * wsz * osz + ci * osz;
            atomicAdd(&d[o0 + ori1], rw1 * cfrac1);
            atomicAdd(&d[o0 + ori2], rw2 * cfrac1);
        }
        if (ci + 1 < wsz) {
            const int o0 = ri * wsz * osz + (ci + 1) * osz;
            atomicAdd(&d[o0 + ori1], rw1 * cfrac);
            atomicAdd(&d[o0 + ori2], rw2 * cfrac);
        }
    }
    if (ri + 1 < wsz) {
        const float rw1 = mag1 * rfrac, rw2 = mag2 * rfrac;
        if (ci >= 0) {
            const int o0 = (ri + 1) * wsz * osz + ci * osz;
            atomicAdd(&d[o0 + ori1], rw1 * cfrac1);
            atomicAdd(&d[o0 + ori2], rw2 * cfrac1);
        }
        if (ci + 1 < wsz) {
            const int o0 = (ri + 1) * wsz * osz + (ci + 1) * osz;
            atomicAdd(&d[o0 + ori1], rw1 * cfrac);
            atomicAdd(&d[o0 + ori2], rw2 * cfrac);
        }
    }
}


struct OriScratch {
    uint64_t bmask[6][72];          // per 64-sample chunk and bin: member samples (bit = t % 64)
    float2 ap[361];                 // (angle, weighted magnitude) per sample: one ds_read_b64
    int   hist[72];
    float avg[72];
    float part[72];
    float pas[84];
    float ws[72];
    float was[72];
};

// assignOrientationApprox (surfd.cu:1711-1960) for one keypoint on one wave.
// lut1: the orientation weights (lookup1, c_tab.lut1 or an LDS copy of it)
__device__ float orientation_wave(const uint32_t* __restrict__ I, const FrameParams& P, const surfhip_point& p,
                                  OriScratch& S, unsigned lane, const float* lut1 = c_tab.lut1)
{
    const int ip = P.ip;
    const DescAt at = ori_at(P.doubled, p);
    const float scale = at.scale;
    const int pixsi = f2i_rz(2.f * scale + 1.6f);
    const int pixsi2 = f2i_rz(scale + 0.8f);
    const int ixo = f2i_rn(at.x), iyo = f2i_rn(at.y);
    for (int t = lane; t < 6 * 72; t += 64) (&S.bmask[0][0])[t] = 0ull;
    wave_sync();
    for (int t = lane; t < 361; t += 64) {
        const int y1 = t / 19 - 9, x1 = t % 19 - 9;
        const int xx = ixo + x1 * pixsi2, yy = iyo + y1 * pixsi2;
        int hid = -1;
        float angle = 0.f, psum = 0.f;
        if (yy + pixsi + 2 < P.iH && yy - pixsi > -1 && xx + pixsi + 2 < P.W + 1 && xx - pixsi > -1) {
            const int distsq = y1 * y1 + x1 * x1;
            if ((float)distsq < 81.5f) {
                const float dx = (float)wavelet2(I, ip, xx, yy, pixsi) * INV255;
                const float dy = (float)wavelet1(I, ip, xx, yy, pixsi) * INV255;
                const float mag = sqrtf(dx * dx + dy * dy);
                if (mag > 0.f) {
                    angle = fast_atan2(dy, dx);
                    hid = f2i_rz((float)(((double)angle + M_PI_D) / (double)SEP_ANGLE_F)) % 72;
                    psum = lut1[distsq] * mag;
                }
            }
        }
        S.ap[t] = make_float2(angle, psum);
        if (hid >= 0) __hip_atomic_fetch_or(&S.bmask[t >> 6][hid], 1ull << (t & 63), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    wave_sync();
    // per-bin sums in row-major sample order (surfd.cu:1820-1840): a bin's
    // lane walks only its member samples, chunk by chunk, bits ascending
    for (int b = lane; b < 72; b += 64) {
        int cnt = 0;
        float sa = 0.f, sp = 0.f, spa = 0.f, swrap = 0.f;
        for (int c = 0; c < 6; c++) {
            uint64_t m = S.bmask[c][b];
            while (m) {
                const int t = 64 * c + (int)__builtin_ctzll(m);
                m &= m - 1;
                const float2 apt = S.ap[t];
                const float a = apt.x, w = apt.y;
                cnt += 1;
                sa = sa + a;
                sp = sp + w;
                spa = spa + a * w;
                if (b < 6) swrap = swrap + (float)(((double)a + 2 * M_PI_D) * (double)w);
                else if (b >= 66) swrap = swrap + (float)(((double)a - 2 * M_PI_D) * (double)w);
            }
        }
        S.hist[b] = cnt;
        S.avg[b] = cnt > 0 ? sa / (float)cnt : c_tab.bins[b];
        S.part[b] = sp;
        S.pas[b + 6] = spa;
        if (b < 6) S.pas[b + 78] = swrap;
        else if (b >= 66) S.pas[b - 66] = swrap;
    }
    wave_sync();
    for (int i = lane; i < 72; i += 64) {
        float ws = 0.f, was = 0.f;
        for (int j = -6; j <= 6; j++) {
            int k = i + j;
            if (j == -6) {
                float residual;
                if (k < 0) {
                    k += 72;
                    const int k1 = (k + 1) % 72;
                    const float t = (c_tab.bins[k1] + (WINDOW_F / 2)) - S.avg[i];
                    residual = (float)((double)t - (c_tab.bins[k1] < 0 ? 0.0 : 2 * M_PI_D));
                } else {
                    residual = (c_tab.bins[k + 1] + (WINDOW_F / 2)) - S.avg[i];
                }
                const float er = residual / SEP_ANGLE_F;
                ws = ws + er * S.part[k];
                was = was + er * S.pas[i];
            } else if (j == 6) {
                float residual;
                if (k >= 72) {
                    k -= 72;
                    const float t = S.avg[i] + (WINDOW_F / 2);
                    residual = (float)(((double)t - 2 * M_PI_D) - (double)c_tab.bins[k]);
                } else {
                    residual = (S.avg[i] + (WINDOW_F / 2)) - c_tab.bins[k];
                }
                const float er = residual / SEP_ANGLE_F;
                ws = ws + er * S.part[k];
                was = was + er * S.pas[i + 12];
            } else {
                was = was + S.pas[k + 6];
                if (k < 0) k += 72;
                else if (k >= 72) k -= 72;
                ws = ws + S.part[k];
            }
        }
        S.ws[i] = ws;
        S.was[i] = was;
    }
    wave_sync();
    // tree argmax in chunks of 64 and 8, strict '<' (surfd.cu:1921-1947):
    // level `stride` updates slots t < stride from t + stride, which that
    // level never writes, so lane-parallel shuffles give the serial result
    float w64 = S.ws[lane], a64 = S.was[lane];
    const int l8 = (int)(lane & 7);
    float w8 = S.ws[64 + l8], a8 = S.was[64 + l8];
#pragma unroll
    for (int stride = 32; stride > 0; stride >>= 1) {
        const float wo = __shfl_down(w64, stride, 64), ao = __shfl_down(a64, stride, 64);
        if ((int)lane < stride && w64 < wo) { w64 = wo; a64 = ao; }
    }
#pragma unroll
    for (int stride = 4; stride > 0; stride >>= 1) {
        const float wo = __shfl_down(w8, stride, 64), ao = __shfl_down(a8, stride, 64);
        if ((int)lane < stride && w8 < wo) { w8 = wo; a8 = ao; }
    }
    float w0 = __shfl(w64, 0, 64), a0 = __shfl(a64, 0, 64);
    const float w1 = __shfl(w8, 0, 64), a1 = __shfl(a8, 0, 64);
    if (w0 < w1) { w0 = w1; a0 = a1; }
    wave_sync();
    return a0 / w0;
}

// XCD-aware keypoint queues for the describe kernels: the workgroups of one
// XCD (blockIdx % 8) take one contiguous eighth of the batch's keypoints (a
// few whole frames, each in the band order k_sort writes), one keypoint per
// grab, so the keypoints in flight on an XCD are consecutive -- a band of a
// frame whose integral-image rows stay in that XCD's L2 (measured on
// k_describe_ur: L2 hit rate 16 % -> 91 %).  The eighth is dealt round-robin
// over kDescQ counters (keypoint gbeg + kDescQ g + q), each on its own 256-B
// line: one same-address atomic per keypoint serialises an XCD at ~50
// cycles a grab.
struct KpQueue {
    int gbeg, gend, qi;
    int* ctr;
    __device__ KpQueue(int total, int* queue, int w)
    {
        const int xcd = blockIdx.x & 7;
        const int chunk = (total + 7) >> 3;
        gbeg = xcd * chunk;
        gend = min(total, gbeg + chunk);
        qi = ((blockIdx.x >> 3) * 4 + w) % kDescQ;
        ctr = queue + (xcd * kDescQ + qi) * 64;
    }
    // the next keypoint (batch index, ascending per wave); >= gend: done
    __device__ int grab(int lane)
    {
        int g = 0;
        if (lane == 0) g = atomicAdd(ctr, 1);
        return gbeg + kDescQ * __builtin_amdgcn_readfirstlane(g) + qi;
    }
    // grab() in two halves: issue the atomic, use its result later
    __device__ int issue(int lane)
    {
        int g = 0;
        if (lane == 0) g = atomicAdd(ctr, 1);
        return g;
    }
    __device__ int finish(int g) { return gbeg + kDescQ * __builtin_amdgcn_readfirstlane(g) + qi; }
};

template <bool UPRIGHT, int MAXF>
__global__ __launch_bounds__(256) void k_describe(const int32_t* __restrict__ ii, FrameParams P,
                                                  surfhip_point* __restrict__ pts, int max_pts,
                                                  const int* __restrict__ counts, const int* __restrict__ offsets,
                                                  const int* __restrict__ order, int nframes, float* __restrict__ desc,
                                                  int* __restrict__ queue)
{
    // four copies of the descriptor per wave (copy = lane & 3, MAXF + 4
    // floats apart so that one bin's copies sit in different banks):
    // neighbouring samples, which mostly hit the same cell and bin, no longer
    // serialise on one LDS address; the copies are summed before
    // normalisation.  MAXF: 128, or 512 for windows past 4 x 4 x 8.
    constexpr int DSTR = MAXF + 4;
    constexpr int NV = MAXF / 64;                // outputs per lane
    __shared__ float sdesc[4][4 * DSTR];
    __shared__ OriScratch sori[UPRIGHT ? 1 : 4];
    const unsigned lane = lane_id();
    const int w = threadIdx.x >> 6;
    const int total = offsets[nframes];
    const int nf = P.nfeat, wsz = P.wsz, osz = P.osz;
    const float fw = (float)wsz;
    const float wofs = (float)wsz * 0.5f - 0.5f;
    float* const d0 = sdesc[w];
    float* d = d0 + (lane & 3) * DSTR;
    KpQueue kq(total, queue, w);
    for (int g = kq.grab((int)lane); g < kq.gend; g = kq.grab((int)lane)) {
        int lo = 0, hi = nframes;            // offsets[lo] <= g < offsets[hi]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (offsets[mid] <= g) lo = mid; else hi = mid;
        }
        const int f = lo, i = order[(size_t)lo * max_pts + (g - offsets[lo])];
        surfhip_point* pp = pts + (size_t)f * max_pts + i;
        const surfhip_point p = *pp;
        const uint32_t* I = reinterpret_cast<const uint32_t*>(ii) + (size_t)f * P.ii_stride;
        const int ip = P.ip;
        float ori = 0.f;
        if constexpr (!UPRIGHT) {
            ori = orientation_wave(I, P, p, sori[w], lane);
            if (lane == 0) pp->ori = ori;
        }
        for (int t = lane; t < 4 * DSTR; t += 64) d0[t] = 0.f;
        wave_sync();
        const DescAt at = desc_at(P.doubled, p);
        const float scale = at.scale;
        const int step = max(f2i_rn(scale * 0.5f), 1);
        const int ix = f2i_rn(at.x), iy = f2i_rn(at.y);
        const float spacing = scale * (float)P.mag;
        const float rspacing = 1.f / spacing;
        const int hs = f2i_rz(scale);
        const int rlim = P.iH - 1 - hs, clim = P.W - hs;   // whps[1].y-1-s, whps[1].x-1-s
        if constexpr (UPRIGHT) {
            const float dx0 = at.x - (float)ix, dy0 = at.y - (float)iy;
            const int iradius = f2i_rn(((spacing * (float)(wsz + 1)) * 0.5f) / (float)step);
            const int side = 2 * iradius + 1;
            const int nsamp = side * side;
            for (int t = lane; t < nsamp; t += 64) {
                const int si = t / side - iradius, sj = t % side - iradius;
                const float rpos = div_by((float)(step * si) - dy0, spacing, rspacing);
                const float cpos = div_by((float)(step * sj) - dx0, spacing, rspacing);
                const float rx = rpos + wofs, cx = cpos + wofs;
                if (!(rx > -1.f && rx < fw && cx > -1.f && cx < fw)) continue;
                const int r = iy + si * step, c = ix + sj * step;
                if (!(r >= 1 + hs && r < rlim && c >= 1 + hs && c < clim)) continue;
                const float weight = c_tab.lut2[f2i_rz(rpos * rpos + cpos * cpos)];
                const float dx = (weight * (float)wavelet2(I, ip, c, r, hs)) * INV255;
                const float dy = (weight * (float)wavelet1(I, ip, c, r, hs)) * INV255;
                if (!P.extend) {
                    place(d, wsz, osz, dx, (dx < 0 ? 0 : 1), dy, (dy < 0 ? 2 : 3), rx, cx);
                } else {
                    place(d, wsz, osz, dx, (dy < 0 ? 0 : 1), fabsf(dx), (dy < 0 ? 2 : 3), rx, cx);
                    place(d, wsz, osz, dy, (dx < 0 ? 4 : 5), fabsf(dy), (dx < 0 ? 6 : 7), rx, cx);
                }
            }
        } else {
            const float fracx = at.x - (float)ix, fracy = at.y - (float)iy;
            const float sine = sincos_poly(ori, 0), cose = sincos_poly(ori, 1);
            const float fracc = ((-sine) * fracy) + (cose * fracx);
            const float fracr = (cose * fracy) + (sine * fracx);
            const int iradius = f2i_rn((((1.4f * spacing) * (float)(wsz + 1)) * 0.5f) / (float)step);
            const int side = 2 * iradius + 1;
            const int nsamp = side * side;
            const float fstep = (float)step;
            for (int t = lane; t < nsamp; t += 64) {
                const int si = t / side - iradius, sj = t % side - iradius;
                const float fi = (float)si, fj = (float)sj;
                const float rpos = div_by((fstep * ((cose * fi) + (sine * fj))) - fracr, spacing, rspacing);
                const float cpos = div_by((fstep * (((-sine) * fi) + (cose * fj))) - fracc, spacing, rspacing);
                const float rx = rpos + wofs, cx = cpos + wofs;
                if (!(rx > -1.f && rx < fw && cx > -1.f && cx < fw)) continue;
                const int r = iy + si * step, c = ix + sj * step;
                if (!(r >= 1 + hs && r < rlim && c >= 1 + hs && c < clim)) continue;
                const float weight = c_tab.lut2[f2i_rz(rpos * rpos + cpos * cpos)];
                const float dxx = (weight * (float)wavelet2(I, ip, c, r, hs)) * INV255;
                const float dyy = (weight * (float)wavelet1(I, ip, c, r, hs)) * INV255;
                const float dx = (cose * dxx) + (sine * dyy);
                const float dy = (sine * dxx) - (cose * dyy);
                if (!P.extend) {
                    place(d, wsz, osz, dx, (dx < 0 ? 0 : 1), dy, (dy < 0 ? 2 : 3), rx, cx);
                } else {
                    place(d, wsz, osz, dx, (dy < 0 ? 0 : 1), fabsf(dx), (dy < 0 ? 2 : 3), rx, cx);
                    place(d, wsz, osz, dy, (dx < 0 ? 4 : 5), fabsf(dy), (dx < 0 ? 6 : 7), rx, cx);
                }
            }
        }
        wave_sync();
        // normalize (surfd.cu:2447-2493): the squares zero-padded to P =
        // max(64, pow2 >= nf) in the sequential-addressing tree: strides P/2
        // .. 64 fold lane + 64 m (m < P / 64) pairwise, then 32 .. 1 across
        // the lanes (for nf = 64 / 128 exactly the reference's order)
        auto sum4 = [&](int b) { return ((d0[b] + d0[DSTR + b]) + d0[2 * DSTR + b]) + d0[3 * DSTR + b]; };
        float v[NV], a2[NV];
#pragma unroll
        for (int m = 0; m < NV; m++) {
            v[m] = (int)lane + 64 * m < nf ? sum4((int)lane + 64 * m) : 0.f;
            a2[m] = v[m] * v[m];
        }
        int np = 1;                                  // P / 64
        while (64 * np < nf) np <<= 1;
#pragma unroll
        for (int half = NV / 2; half >= 1; half >>= 1)
            if (half < np)
#pragma unroll
                for (int m = 0; m < half; m++) a2[m] = a2[m] + a2[m + half];
        float a = a2[0];
#pragma unroll
        for (int k = 32; k >= 1; k >>= 1) a = a + __shfl_down(a, k, 64);
        const float tot = __shfl(a, 0, 64);
        const float fac = 1.f / sqrtf(tot);
        float* out = desc + ((size_t)f * max_pts + i) * nf;
#pragma unroll
        for (int m = 0; m < NV; m++)
            if ((int)lane + 64 * m < nf) out[lane + 64 * m] = v[m] * fac;
        wave_sync();
    }
}

// ----------------------------------------------------------------------
// Rotated descriptor without atomics (wsz = 4; 64-D or 128-D extended).
// The rotated window's sample grid (surfd.cu:2391-2444) is not separable,
// but each sample adds only into the 2 x 2 cells at its floor cell (ri, ci)
// (placeInIndex, surfd.cu:1199-1271).  So a lane pair owns one floor cell
// of the 5 x 5 set {-1..3}^2: it walks the grid samples inside a
// conservative bounding box of that cell's rotated square (the inverse
// rotation of its corners, one sample of slack), keeps exactly the samples
// whose floor cell -- computed with the reference's float ops -- is its own
// (so every sample is counted once), and accumulates the 4 cells x NB bins
// it can touch in registers.  A fixed-order sum over the (at most 8)
// contributing lanes of each output bin replaces the LDS float atomics,
// so the descriptor is deterministic.  Orientation as k_describe.
// ----------------------------------------------------------------------
struct RotScratch {
    union {
        OriScratch ori;
        float red[64][4 * 8 + 1];   // per lane: 4 relative cells x NB bins (+1 pad)
    };
};

#ifndef SURF_ROT_LDS_LUT
#define SURF_ROT_LDS_LUT 1
#endif
#ifndef SURF_ROT_WPE
#define SURF_ROT_WPE 3              // 3 waves per SIMD: <= 168 VGPRs (the 128-D form took 185: 2 waves)
#endif
template <int NB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SURF_ROT_WPE))) void k_describe_rot(const int32_t* __restrict__ ii, FrameParams P,
                                                      surfhip_point* __restrict__ pts, int max_pts,
                                                      const int* __restrict__ offsets, const int* __restrict__ order,
                                                      int nframes, float* __restrict__ desc, int* __restrict__ queue)
{
    constexpr int WSZ = 4, NC = WSZ + 1, NF = WSZ * WSZ * NB;
    __shared__ RotScratch sr[4];
#if SURF_ROT_LDS_LUT
    // the Gaussian weight tables in LDS: each sample's weight is one
    // lane-indexed read, from LDS instead of a global load on the walk's
    // dependency chain (same values)
    __shared__ float s_lut1[83], s_lut2[40];
    for (int t = threadIdx.x; t < 83; t += blockDim.x) s_lut1[t] = c_tab.lut1[t];
    for (int t = threadIdx.x; t < 40; t += blockDim.x) s_lut2[t] = c_tab.lut2[t];
    __syncthreads();
    const float* const lut1 = s_lut1;
    const float* const lut2 = s_lut2;
#else
    const float* const lut1 = c_tab.lut1;
    const float* const lut2 = c_tab.lut2;
#endif
    const unsigned lane = lane_id();
    const int w = threadIdx.x >> 6;
    const int total = offsets[nframes];
    const float fw = (float)WSZ;
    const float wofs = (float)WSZ * 0.5f - 0.5f;
    // this lane's floor cell (lanes 50..63 own none)
    const int cidx = (int)lane >> 1, half = (int)lane & 1;
    const bool owner = cidx < NC * NC;
    const int cri = owner ? cidx / NC - 1 : -100, cci = owner ? cidx % NC - 1 : -100;
    RotScratch& S = sr[w];
    KpQueue kq(total, queue, w);
    for (int g = kq.grab((int)lane); g < kq.gend; g = kq.grab((int)lane)) {
        int lo = 0, hi = nframes;            // offsets[lo] <= g < offsets[hi]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (offsets[mid] <= g) lo = mid; else hi = mid;
        }
        const int f = lo, i = order[(size_t)lo * max_pts + (g - offsets[lo])];
        surfhip_point* pp = pts + (size_t)f * max_pts + i;
        const surfhip_point p = *pp;
        const uint32_t* I = reinterpret_cast<const uint32_t*>(ii) + (size_t)f * P.ii_stride;
        const int ip = P.ip;
#ifdef SURF_DIAG_NOORI
        const float ori = 0.3f;
#else
        const float ori = orientation_wave(I, P, p, S.ori, lane, lut1);
#endif
        if (lane == 0) pp->ori = ori;
#ifdef SURF_DIAG_NODESC
        if (lane < 2) desc[((size_t)f * max_pts + i) * NF + lane] = ori;
        continue;
#endif

        const DescAt at = desc_at(P.doubled, p);
        const float scale = at.scale;
        const int step = max(f2i_rn(scale * 0.5f), 1);
        const int ix = f2i_rn(at.x), iy = f2i_rn(at.y);
        const float spacing = scale * (float)P.mag;
        const int hs = f2i_rz(scale);
        const int rlim = P.iH - 1 - hs, clim = P.W - hs;
        const float fracx = at.x - (float)ix, fracy = at.y - (float)iy;
        const float sine = sincos_poly(ori, 0), cose = sincos_poly(ori, 1);
        const float fracc = ((-sine) * fracy) + (cose * fracx);
        const float fracr = (cose * fracy) + (sine * fracx);
        const int iradius = f2i_rn((((1.4f * spacing) * (float)(WSZ + 1)) * 0.5f) / (float)step);
        const float fstep = (float)step;
        const float rspacing = 1.f / spacing;
        // grid box of this lane's cell: inverse rotation of its corners
        int i0 = 1, i1 = 0, j0 = 0, j1 = 0;
        if (owner) {
            float mni = 1e30f, mxi = -1e30f, mnj = 1e30f, mxj = -1e30f;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const float A = ((float)(cri + (k >> 1)) - wofs) * spacing + fracr;
                const float B = ((float)(cci + (k & 1)) - wofs) * spacing + fracc;
                const float fi = (cose * A - sine * B) / fstep, fj = (sine * A + cose * B) / fstep;
                mni = fminf(mni, fi); mxi = fmaxf(mxi, fi);
                mnj = fminf(mnj, fj); mxj = fmaxf(mxj, fj);
            }
#ifdef SURF_ROT_LOOSE
            i0 = max(-iradius, (int)floorf(mni) - 1);
            i1 = min(iradius, (int)ceilf(mxi) + 1);
            j0 = max(-iradius, (int)floorf(mnj) - 1);
            j1 = min(iradius, (int)ceilf(mxj) + 1);
#else
            // the integer rows / columns inside the box, widened by kSlackBox
            // (the corners' float error is far below it; membership is the
            // exact test below).  Rounding outwards and a sample more on each
            // side walked 2 empty rows per lane (tools/rot_walk_count.py)
            constexpr float kSlackBox = 0.05f;
            i0 = max(-iradius, (int)ceilf(mni - kSlackBox));
            i1 = min(iradius, (int)floorf(mxi + kSlackBox));
            j0 = max(-iradius, (int)ceilf(mnj - kSlackBox));
            j1 = min(iradius, (int)floorf(mxj + kSlackBox));
#endif
            i0 += half;                      // the pair splits the box rows by parity
        }
        // per box row, the sj interval where the cell's two slabs (rx in
        // [cri, cri + 1], cx in [cci, cci + 1]) cross the row, widened by
        // kSlack samples (the inverse's float error is < 1e-2 samples for
        // slopes >= 1e-3; membership itself is the exact test below); a
        // near-zero slope keeps the whole box row
        constexpr float kSlack = 0.05f;
        const float Alo = (((float)cri - wofs) * spacing + fracr) / fstep;
        const float Ahi = (((float)(cri + 1) - wofs) * spacing + fracr) / fstep;
        const float Blo = (((float)cci - wofs) * spacing + fracc) / fstep;
        const float Bhi = (((float)(cci + 1) - wofs) * spacing + fracc) / fstep;
        const bool use_s = fabsf(sine) > 1e-3f, use_c = fabsf(cose) > 1e-3f;
        const float inv_s = use_s ? 1.f / sine : 0.f, inv_c = use_c ? 1.f / cose : 0.f;
        int rlo = 0, rhi = -1;
        auto row_range = [&](int row) {
            const float fi = (float)row;
            float lo = (float)j0, hi = (float)j1;
            if (use_s) {                     // sine * fj in [Alo - cose fi, Ahi - cose fi]
                const float a = (Alo - cose * fi) * inv_s, b = (Ahi - cose * fi) * inv_s;
                lo = fmaxf(lo, fminf(a, b) - kSlack);
                hi = fminf(hi, fmaxf(a, b) + kSlack);
            }
            if (use_c) {                     // cose * fj in [Blo + sine fi, Bhi + sine fi]
                const float a = (Blo + sine * fi) * inv_c, b = (Bhi + sine * fi) * inv_c;
                lo = fmaxf(lo, fminf(a, b) - kSlack);
                hi = fminf(hi, fmaxf(a, b) + kSlack);
            }
#ifdef SURF_ROT_LOOSE
            rlo = (int)floorf(lo);
            rhi = (int)ceilf(hi);
#else
            // the integers inside [lo, hi] (already widened by kSlack):
            // rounded outwards, a third of the samples walked were rejected
            // by the membership test (tools/rot_walk_count.py: 1,349 walked
            // for 900 members per keypoint, 925 rounded inwards)
            rlo = (int)ceilf(lo);
            rhi = (int)floorf(hi);
#endif
            rlo = max(rlo, j0);
            rhi = min(rhi, j1);
        };
        // relative cells q = 0..3 ({(0,0), (0,1), (1,0), (1,1)} from the floor
        // cell) in pairs: accp[h][b] = {cell 2h, cell 2h + 1} of bin b
        v2f32 accp[2][NB];
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
            for (int b = 0; b < NB; b++) accp[h][b] = v2f32{0.f, 0.f};
        int si = i0, sj = 0;
        if (si <= i1) { row_range(si); sj = rlo; }
        while (si <= i1) {
            if (sj > rhi) {
                si += 2;
                if (si <= i1) { row_range(si); sj = rlo; }
                continue;
            }
            const int cj = sj++;
            const float fi = (float)si, fj = (float)cj;
            // the IEEE quotient as the reference: rpos^2 + cpos^2 indexes the
            // Gaussian LUT, so one ulp can move a sample to the next weight
            // (x * (1 / spacing) alone broke config #5 parity at 1.3e-3 L2);
            // div_by is exact where it matters
            const float rpos = div_by((fstep * ((cose * fi) + (sine * fj))) - fracr, spacing, rspacing);
            const float cpos = div_by((fstep * (((-sine) * fi) + (cose * fj))) - fracc, spacing, rspacing);
            const float rx = rpos + wofs, cx = cpos + wofs;
            if (!(rx > -1.f && rx < fw && cx > -1.f && cx < fw)) continue;
            const int ri = f2i_rz(rx >= 0.f ? rx : rx - 1.f);
            const int ci = f2i_rz(cx >= 0.f ? cx : cx - 1.f);
            if (ri != cri || ci != cci) continue;
            const int r = iy + si * step, c = ix + cj * step;
            if (!(r >= 1 + hs && r < rlim && c >= 1 + hs && c < clim)) continue;
            const float weight = lut2[f2i_rz(rpos * rpos + cpos * cpos)];
#ifdef SURF_DIAG_ROT_NOLOAD
            const float dxx = (weight * (float)(r * 7 - c)) * INV255;
            const float dyy = (weight * (float)(c * 3 + r)) * INV255;
#else
            const float dxx = (weight * (float)wavelet2(I, ip, c, r, hs)) * INV255;
            const float dyy = (weight * (float)wavelet1(I, ip, c, r, hs)) * INV255;
#endif
            const float dx = (cose * dxx) + (sine * dyy);
            const float dy = (sine * dxx) - (cose * dyy);
            const float rfrac = rx - (float)ri, cfrac = cx - (float)ci;
            const float cfrac1 = 1 - cfrac;
            const float rfrac1 = 1.f - rfrac;
            const v2f32 cw = {cfrac1, cfrac};
            // placeInIndex products (surfd.cu:1222-1266): cell weight by row,
            // then column -- {r0, r0} * {cfrac1, cfrac} is the reference's two
            // products of row ri in one packed multiply.  One placeInIndex
            // value goes to bin BN when `neg`, else BP (both static): a packed
            // FMA by 1 or 0 adds it exactly (v * 1 + acc rounds once, as acc +
            // v; v * 0 + acc = acc), 4 packed FMAs for the 4 cells x 2 bins
            // instead of 8 selects and 8 adds (the kernel's time did not move:
            // it waits on its gathers)
            auto put = [&](auto bn, auto bp, float mag, bool neg) {
                constexpr int BN = decltype(bn)::value, BP = decltype(bp)::value;
                const float r0 = mag * rfrac1, r1 = mag * rfrac;
                const v2f32 v01 = v2f32{r0, r0} * cw, v23 = v2f32{r1, r1} * cw;
                const float mn = neg ? 1.f : 0.f, mp = neg ? 0.f : 1.f;
                const v2f32 n2 = {mn, mn}, p2 = {mp, mp};
                accp[0][BN] = __builtin_elementwise_fma(v01, n2, accp[0][BN]);
                accp[1][BN] = __builtin_elementwise_fma(v23, n2, accp[1][BN]);
                accp[0][BP] = __builtin_elementwise_fma(v01, p2, accp[0][BP]);
                accp[1][BP] = __builtin_elementwise_fma(v23, p2, accp[1][BP]);
            };
            using I0 = std::integral_constant<int, 0>;
            using I1 = std::integral_constant<int, 1>;
            using I2 = std::integral_constant<int, 2>;
            using I3 = std::integral_constant<int, 3>;
            if constexpr (NB == 4) {
                put(I0{}, I1{}, dx, dx < 0);
                put(I2{}, I3{}, dy, dy < 0);
            } else {
                using I4 = std::integral_constant<int, 4>;
                using I5 = std::integral_constant<int, 5>;
                using I6 = std::integral_constant<int, 6>;
                using I7 = std::integral_constant<int, 7>;
                put(I0{}, I1{}, dx, dy < 0);
                put(I2{}, I3{}, fabsf(dx), dy < 0);
                put(I4{}, I5{}, dy, dx < 0);
                put(I6{}, I7{}, fabsf(dy), dx < 0);
            }
        }
        wave_sync();                          // orientation scratch is dead: reuse it
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
            for (int b = 0; b < NB; b++) S.red[lane][q * NB + b] = (q & 1) ? accp[q >> 1][b].y : accp[q >> 1][b].x;
        wave_sync();
        // output bin (R, C, b): floor cells (R, C), (R, C-1), (R-1, C), (R-1, C-1)
        // via relative cells 0..3, each by its two lanes, in that fixed order
        float vout[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int o = (int)lane + 64 * h;
            float a = 0.f;
            if (o < NF) {
                const int cell = o / NB, b = o % NB, R = cell / WSZ, C = cell % WSZ;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int fr = R - (q >> 1), fc = C - (q & 1);      // floor cell of the contributors
                    const int fl = ((fr + 1) * NC + (fc + 1)) * 2;
                    a = a + S.red[fl][q * NB + b];
                    a = a + S.red[fl + 1][q * NB + b];
                }
            }
            vout[h] = a;
        }
        // normalize (surfd.cu:2447-2493)
        float a2 = vout[0] * vout[0];
        if (NF > 64) a2 = a2 + vout[1] * vout[1];
#pragma unroll
        for (int k = 32; k >= 1; k >>= 1) a2 = a2 + __shfl_down(a2, k, 64);
        const float tot = __shfl(a2, 0, 64);
        const float fac = 1.f / sqrtf(tot);
        float* out = desc + ((size_t)f * max_pts + i) * NF;
        out[lane] = vout[0] * fac;
        if (NF > 64) out[lane + 64] = vout[1] * fac;
        wave_sync();
    }
}

// ----------------------------------------------------------------------
// Upright descriptor (U-SURF, 4x4 cells), deterministic and atomic-free.
// The upright sample grid is separable (surfd.cu:1290-1294): a sample's cell
// row (ri, rfrac) depends only on its grid row i, its cell column (ci, cfrac)
// only on its grid column j.  So:
//  * lane = grid column j; when the grid is at most 32 columns wide (iradius
//    <= 15, ~2/3 of keypoints) the two half-waves walk alternate grid rows,
//    so no lane idles on the wide-grid padding;
//  * the rows are walked in cell-row bands (ri = -1..3, contiguous because ri
//    is monotonic in i), each band compile-time, so the placeInIndex row
//    weights (1 - rfrac, rfrac) go into fixed registers: per band a lane keeps
//    P = sum v and Q = sum v * rfrac, then row ri gets P - Q and row ri + 1
//    gets Q (surfd.cu:1199-1271 with the sums regrouped);
//  * bins are kept as (total, negative part) pairs, so the sign-selected
//    bins cost a min/select instead of a branch;
//  * the column weights (1 - cfrac, cfrac) are applied once per lane in a
//    fixed-order reduction over the lanes of each cell column.
// Grid-row geometry (rpos, rx, ri, rfrac) is computed once per row, with the
// reference's exact float operations, so cell membership and the lookup2
// index match the oracle bit for bit; only the summation order differs
// (<= 1e-6 relative, inside the 1e-4 descriptor tolerance).
// Integral-image reads are raw buffer loads (SGPR descriptor + 32-bit
// offsets, no 64-bit address arithmetic).  iradius <= 22 for wsz 4, so the
// grid fits one wave.
// ----------------------------------------------------------------------
__device__ __forceinline__ __amdgpu_buffer_rsrc_t frame_rsrc(const uint32_t* I, long long nbytes)
{
    return __builtin_amdgcn_make_buffer_rsrc((void*)I, (short)0, (int)nbytes, 0x00020000);
}
__device__ __forceinline__ uint32_t bld(__amdgpu_buffer_rsrc_t r, int off)
{
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}

template <int NS>
__device__ __forceinline__ void haar_bins(int32_t wav1, int32_t wav2, float weight, bool ok, float (&S)[NS])
{
    // {dx, dy} = weight * {wav2, wav1} in one packed multiply; a lane
    // outside the grid contributes 0 (a select: its inputs may be garbage)
    v2f32 d = v2f32{(float)wav2, (float)wav1} * weight;
    const float dx = ok ? d.x : 0.f, dy = ok ? d.y : 0.f;
    if constexpr (NS == 4) {
        S[0] = dx; S[1] = fminf(dx, 0.f);          // bins 1 | 0 by sign of dx
        S[2] = dy; S[3] = fminf(dy, 0.f);          // bins 3 | 2 by sign of dy
    } else {
        const float adx = fabsf(dx), ady = fabsf(dy);
        S[0] = dx;  S[1] = dy < 0.f ? dx : 0.f;    // bins 1 | 0 by sign of dy
        S[2] = adx; S[3] = dy < 0.f ? adx : 0.f;   // bins 3 | 2
        S[4] = dy;  S[5] = dx < 0.f ? dy : 0.f;    // bins 5 | 4 by sign of dx
        S[6] = ady; S[7] = dx < 0.f ? ady : 0.f;   // bins 7 | 6
    }
}

template <int R> struct IntC { static constexpr int value = R; };

// value of lane - 2 / lane + 2 across the whole wave (DPP wave_shr:1 /
// wave_shl:1 twice; lanes shifted in from outside the wave get 0)
__device__ __forceinline__ uint32_t wave_from_lo2(uint32_t v)
{
    const int a = __builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
    return (uint32_t)__builtin_amdgcn_update_dpp(0, a, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_from_hi2(uint32_t v)
{
    const int a = __builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);
    return (uint32_t)__builtin_amdgcn_update_dpp(0, a, 0x130, 0xf, 0xf, false);
}

template <bool EXT>
__global__ __launch_bounds__(256) void k_describe_ur(const int32_t* __restrict__ ii, FrameParams P,
                                                     const surfhip_point* __restrict__ pts, int max_pts,
                                                     const int* __restrict__ offsets,
                                                     const int* __restrict__ order, int nframes,
                                                     float* __restrict__ desc, int* __restrict__ queue)
{
    constexpr int WSZ = 4;
    constexpr int NB = EXT ? 8 : 4;                       // bins per cell
    constexpr int NF = WSZ * WSZ * NB;
    constexpr int RS = WSZ * NB + 1;                      // odd stride: conflict-free writes
    __shared__ float red[4][64][RS];
    __shared__ float s_cf[4][64];
    __shared__ float s_rf[4][64], s_rp[4][64];
    __shared__ int s_ri[4][64];
    __shared__ float4 s_wr[4][64];               // per grid row: weights of cell rows 0..3
    __shared__ __attribute__((aligned(16))) uint32_t s_seg[4][448];   // segment path: the wave's integral rows
    __shared__ int4 s_run[4][6];
    // Gaussian weights premultiplied by 1/255 (the reference scales the Haar
    // response by the weight, then by 1/255: one rounding moves, within the
    // descriptor tolerance)
    __shared__ float s_lut[40];
    if (threadIdx.x < 40) s_lut[threadIdx.x] = c_tab.lut2[threadIdx.x] * INV255;
    __syncthreads();
    const int lane = (int)lane_id();
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);     // wave-uniform: SGPR descriptors
    const int total = offsets[nframes];
    const float fw = (float)WSZ;
    const float wofs = (float)WSZ * 0.5f - 0.5f;
    KpQueue kq(total, queue, w);
    const int gend = kq.gend;
    auto grab = [&]() { return kq.grab(lane); };
    // the wave's keypoints ascend, so its frame is tracked incrementally
    // (one binary search per wave) and the next keypoint is fetched while
    // the current one is described
    int gn = grab();
    int fn = 0, fnb = 0, fne = 0, kn = 0;
    surfhip_point pn;
    if (gn < gend) {
        int lo = 0, hi = nframes;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (offsets[mid] <= gn) lo = mid; else hi = mid;
        }
        fn = lo;
        fnb = offsets[lo];
        fne = offsets[lo + 1];
        kn = order[(size_t)fn * max_pts + (gn - fnb)];
        pn = pts[(size_t)fn * max_pts + kn];
    }
    while (gn < gend) {
        const int f = fn, kp = kn;
        const surfhip_point p = pn;
        gn = grab();
        if (gn < gend) {
            while (gn >= fne) { fn++; fnb = fne; fne = offsets[fn + 1]; }
            kn = order[(size_t)fn * max_pts + (gn - fnb)];
            pn = pts[(size_t)fn * max_pts + kn];
        }
        const uint32_t* I = reinterpret_cast<const uint32_t*>(ii) + (size_t)f * P.ii_stride;
        const __amdgpu_buffer_rsrc_t rsrc = frame_rsrc(I, P.ii_stride * 4);
        const DescAt at = desc_at(P.doubled, p);
        const float scale = at.scale;
        const int step = max(f2i_rn(scale * 0.5f), 1);
        const int ix = f2i_rn(at.x), iy = f2i_rn(at.y);
        const float dx0 = at.x - (float)ix, dy0 = at.y - (float)iy;
        const float spacing = scale * (float)P.mag;
        const int hs = f2i_rz(scale);
        const int rlim = P.iH - 1 - hs, clim = P.W - hs;
        const int iradius = f2i_rn(((spacing * (float)(WSZ + 1)) * 0.5f) / (float)step);
        const int side = 2 * iradius + 1;
        // ---- grid row t = lane: exact row geometry (surfd.cu:1290-1292)
        const int sit = lane - iradius;
        const float rpos_t = ((float)(step * sit) - dy0) / spacing;
        const float rx_t = rpos_t + wofs;
        const int r_t = iy + sit * step;
        const bool rvalid = lane < side && rx_t > -1.f && rx_t < fw && r_t >= 1 + hs && r_t < rlim;
        const int ri_t = f2i_rz(rx_t >= 0.f ? rx_t : rx_t - 1.f);
        s_rf[w][lane] = rx_t - (float)ri_t;
        s_rp[w][lane] = rpos_t * rpos_t;
        s_ri[w][lane] = ri_t;
        {
            // placeInIndex's row weights (surfd.cu:1199-1271): 1 - rfrac for
            // cell row ri, rfrac for ri + 1
            const float rf_t = rx_t - (float)ri_t, w0_t = 1.f - rf_t;
            s_wr[w][lane] = make_float4(ri_t == 0 ? w0_t : (ri_t == -1 ? rf_t : 0.f),
                                        ri_t == 1 ? w0_t : (ri_t == 0 ? rf_t : 0.f),
                                        ri_t == 2 ? w0_t : (ri_t == 1 ? rf_t : 0.f),
                                        ri_t == 3 ? w0_t : (ri_t == 2 ? rf_t : 0.f));
        }
        // ---- grid column of this lane (lane = j; dual: two half-waves of 32
        // lanes walk alternate grid rows)
        const int hmode = hs - 2 * step;          // 0 or -1: rows and columns share integral pairs
        const bool share = hmode == 0 || hmode == -1;
        const bool dual = side <= 32;
        const int j = dual ? (lane & 31) : lane;
        const int h = dual ? (lane >> 5) : 0;
        const int rstep = dual ? 2 : 1;
        const int sj = j - iradius;
        const float cpos = ((float)(step * sj) - dx0) / spacing;
        const float cx = cpos + wofs;
        const int c = ix + sj * step;
        const bool col_on = j < side && cx > -1.f && cx < fw && c >= 1 + hs && c < clim;
        const int ci = f2i_rz(cx >= 0.f ? cx : cx - 1.f);
        const float cfrac = cx - (float)ci;
        const float cp2 = cpos * cpos;
        const int ip4 = P.ip * 4;
        const int oA = (c - hs) * 4, oB = (c + hs + 1) * 4, oC = c * 4;
        const int dR0 = -hs * ip4, dR3 = (hs + 1) * ip4;
        wave_sync();
        constexpr int NS = EXT ? 8 : 4;
        float acc[WSZ][NS];
#pragma unroll
        for (int R = 0; R < WSZ; R++)
#pragma unroll
            for (int s = 0; s < NS; s++) acc[R][s] = 0.f;
        // ---- the valid grid rows form one contiguous run [t0, t0 + nv); half h
        // takes rows t0 + h, t0 + h + rstep, ...
        // A row adds S * (1 - rfrac) to cell row ri and S * rfrac to ri + 1
        // (placeInIndex, surfd.cu:1199-1271); the weights of the 4 cell rows
        // are formed by selects, so the accumulators keep fixed registers.
        const unsigned long long vm = __ballot(rvalid);
        const int t0 = vm ? __builtin_ctzll(vm) : 0, nv = __builtin_popcountll(vm);
        // one sample: its 12 integral-image corners -> haar responses -> bins
        auto accum = [&](uint32_t a00, uint32_t a01, uint32_t a02, uint32_t a03, uint32_t a10, uint32_t a11,
                         uint32_t a20, uint32_t a21, uint32_t a30, uint32_t a31, uint32_t a32, uint32_t a33,
                         int tt) {
            const float rf = s_rf[w][tt];
            const float rp = s_rp[w][tt];
            const int ri = s_ri[w][tt];
            // haarX / haarY (surfd.cu:1171-1182 via getSum); rows r-s, r, r+1,
            // r+s+1 (a0*, a1*, a2*, a3*), cols c-s, c+s+1, c, c+1
            const int32_t wav1 = (int32_t)((a21 + a00 - a01 - a20) - (a31 + a10 - a11 - a30));
            const int32_t wav2 = (int32_t)((a31 + a02 - a01 - a32) - (a33 + a00 - a03 - a30));
            float S[NS];
            haar_bins(wav1, wav2, s_lut[f2i_rz(rp + cp2)], true, S);
            const float w0 = 1.f - rf;
            // the cell row is uniform over the wave except where the two
            // halves (dual mode) straddle a cell-row boundary
            const int riu = __builtin_amdgcn_readfirstlane(ri);
            if (__all(ri == riu)) {
#pragma unroll
                for (int R = 0; R < WSZ; R++) {
                    if (R == riu) {
#pragma unroll
                        for (int s = 0; s < NS; s++) acc[R][s] = fmaf(S[s], w0, acc[R][s]);
                    } else if (R == riu + 1) {
#pragma unroll
                        for (int s = 0; s < NS; s++) acc[R][s] = fmaf(S[s], rf, acc[R][s]);
                    }
                }
            } else {
#pragma unroll
                for (int R = 0; R < WSZ; R++) {
                    const float rw = (R == ri) ? w0 : ((R == ri + 1) ? rf : 0.f);
#pragma unroll
                    for (int s = 0; s < NS; s++) acc[R][s] = fmaf(S[s], rw, acc[R][s]);
                }
            }
        };
        if (share) {
            // ---- Row and column sharing.  step = rn(scale / 2) and hs =
            // rz(scale) give hs = 2 step or 2 step - 1, so the outer rows
            // r - hs and r + hs + 1 of grid row i are rows r and r + 1 of grid
            // rows i - 2 and i + 2, and likewise the columns.  Each half walks
            // every other grid row (dual: rows of its parity; single: even
            // rows, then odd rows).  Per integral row a lane loads its (c, c+1)
            // pair (8 bytes, issued three grid rows ahead into a raw slot);
            // when the row is first needed it takes columns c - hs and
            // c + hs + 1 from lanes j -+ 2, except the two edge lanes on each
            // side, which load that column themselves (the same instruction,
            // every other lane past the buffer).  4 loads per sample (was 12).
            const bool ld_on = j < side;
            const bool eL = j < 2, eR = j + 2 >= side;
            const int oE = eL ? oA : oB;          // edge lanes: c - hs (left) / c + hs + 1 (right)
            const int nph = dual ? 1 : 2;
            struct Raw { v2u32 lo, hi; uint32_t elo, ehi; };
            auto ldraw = [&](int t) {
                const int rb = (iy + (t - iradius) * step) * ip4;
                const int o = ld_on ? rb + oC : (int)kOOB;
                const int oe = (ld_on && (eL || eR)) ? rb + oE : (int)kOOB;
                Raw q;
#ifdef SURF_DIAG_NOLOAD
                q.lo = v2u32{(uint32_t)o, (uint32_t)o + 7u};
                q.hi = v2u32{(uint32_t)o * 3u, (uint32_t)o + 11u};
                q.elo = (uint32_t)oe;
                q.ehi = (uint32_t)oe * 5u;
#elif defined(SURF_DIAG_NOEDGE)
                q.lo = __builtin_amdgcn_raw_buffer_load_b64(rsrc, o, 0, 0);
                q.hi = __builtin_amdgcn_raw_buffer_load_b64(rsrc, ld_on ? o + ip4 : (int)kOOB, 0, 0);
                q.elo = (uint32_t)oe;
                q.ehi = (uint32_t)oe * 5u;
#else
                q.lo = __builtin_amdgcn_raw_buffer_load_b64(rsrc, o, 0, 0);
                q.hi = __builtin_amdgcn_raw_buffer_load_b64(rsrc, ld_on ? o + ip4 : (int)kOOB, 0, 0);
                q.elo = bld(rsrc, oe);
                q.ehi = bld(rsrc, (ld_on && (eL || eR)) ? oe + ip4 : (int)kOOB);
#endif
                return q;
            };
            // The row loop, specialised on hmode (A: hs = 2 step).  A row adds
            // S (1 - rfrac) to cell row ri and S rfrac to ri + 1: the four
            // row weights come precomputed per grid row (s_wr).
            auto rows = [&](auto AC) {
                constexpr bool A = decltype(AC)::value;
                // T = rows r, r+1 x cols c-s, c, c+1, c+s+1
                // columns c -+ hs from lanes j -+ 2: two DPP wave shifts each
                // (VALU) instead of an LDS permute
                auto proc = [&](const Raw& q, uint32_t (&T)[8]) {
                    T[1] = q.lo.x; T[2] = q.lo.y; T[5] = q.hi.x; T[6] = q.hi.y;
                    const uint32_t l0 = wave_from_lo2(A ? q.lo.x : q.lo.y);
                    const uint32_t r0 = wave_from_hi2(A ? q.lo.y : q.lo.x);
                    const uint32_t l1 = wave_from_lo2(A ? q.hi.x : q.hi.y);
                    const uint32_t r1 = wave_from_hi2(A ? q.hi.y : q.hi.x);
                    T[0] = eL ? q.elo : l0;
                    T[3] = eR ? q.elo : r0;
                    T[4] = eL ? q.ehi : l1;
                    T[7] = eR ? q.ehi : r1;
                };
                for (int ph = 0; ph < nph; ph++) {
                    const int hh = dual ? h : ph;
                    // rows t0 + hh, t0 + hh + 2, ...: nstep of them (the halves
                    // of a dual wave may differ by one; the loop runs the larger)
                    const int nstep = max(nv - hh + 1, 0) >> 1;
                    const int nmax = dual ? max(nv + 1, 0) >> 1 : nstep;
                    if (nmax == 0) continue;
#ifdef SURF_DIAG_NOROWS
                    continue;
#endif
                    // one sample of grid row t from the sets of rows t - 2, t, t + 2
                    auto sample = [&](int n, const uint32_t (&Pv)[8], const uint32_t (&Cv)[8],
                                      const uint32_t (&Nv)[8]) {
                        const int t = t0 + hh + 2 * n;
                        if (!(col_on && n < nstep)) return;
                        constexpr bool ok = true;
#ifdef SURF_DIAG_NOCOMP
                        acc[0][0] += (float)(Pv[0] ^ Cv[3] ^ Nv[5] ^ Pv[7] ^ Nv[1]);
                        return;
#endif
                        const float rp = s_rp[w][t];
                        const float4 wr = s_wr[w][t];
                        // top row r - hs, bottom row r + hs + 1; rows r-s, r, r+1,
                        // r+s+1 (a0*, a1*, a2*, a3*), cols c-s, c+s+1, c, c+1
                        const uint32_t a00 = A ? Pv[0] : Pv[4], a02 = A ? Pv[1] : Pv[5];
                        const uint32_t a03 = A ? Pv[2] : Pv[6], a01 = A ? Pv[3] : Pv[7];
                        const uint32_t a30 = A ? Nv[4] : Nv[0], a32 = A ? Nv[5] : Nv[1];
                        const uint32_t a33 = A ? Nv[6] : Nv[2], a31 = A ? Nv[7] : Nv[3];
                        const uint32_t a10 = Cv[0], a11 = Cv[3], a20 = Cv[4], a21 = Cv[7];
                        // haarX / haarY (surfd.cu:1171-1182 via getSum)
                        const int32_t wav1 = (int32_t)((a21 + a00 - a01 - a20) - (a31 + a10 - a11 - a30));
                        const int32_t wav2 = (int32_t)((a31 + a02 - a01 - a32) - (a33 + a00 - a03 - a30));
                        float S[NS];
                        haar_bins(wav1, wav2, s_lut[f2i_rz(rp + cp2)], ok, S);
                        // all four cell rows with the row's weights (two are 0):
                        // branch-free, fixed registers
                        const float wrr[WSZ] = {wr.x, wr.y, wr.z, wr.w};
#pragma unroll
                        for (int R = 0; R < WSZ; R++)
#pragma unroll
                            for (int e = 0; e < NS; e++) acc[R][e] = fmaf(S[e], wrr[R], acc[R][e]);
                    };
                    // 8-value sets X, Y, Z rotate through the roles (top, middle,
                    // bottom) and raw slots s0..s2 hold the rows 2, 4, 6 ahead;
                    // unrolled by 3 so no register moves the sets around.  All
                    // loads are unconditional (past the buffer where not needed),
                    // so hipcc's outstanding-load count stays exact.
                    uint32_t X[8], Y[8], Z[8];
                    const int tb = t0 + hh;
                    const Raw q0 = ldraw(tb - 2), q1 = ldraw(tb);
                    Raw s0 = ldraw(tb + 2), s1 = ldraw(tb + 4), s2 = ldraw(tb + 6);
                    proc(q0, X);
                    proc(q1, Y);
                    for (int n = 0; n < nmax; n += 3) {
                        const int t = tb + 2 * n;
                        proc(s0, Z);
                        s0 = ldraw(t + 8);
                        sample(n, X, Y, Z);
                        proc(s1, X);
                        s1 = ldraw(t + 10);
                        sample(n + 1, Y, Z, X);
                        proc(s2, Y);
                        s2 = ldraw(t + 12);
                        sample(n + 2, Z, X, Y);
                    }
                }
            };
            // ---- segment path (step <= 3, ~80 % of keypoints): the needed
            // columns c_j - hs .. c_j + hs + 1 of all grid columns tile one
            // contiguous span of each integral row, so a wave step loads the
            // span of its 2 (dual: 4) integral rows as 16-byte chunks (1-2
            // instructions instead of 4), stages them in a per-wave LDS row
            // buffer and every lane reads its 8 values from there.
            const int G = dual ? 2 : 1;
            const int cs = (ix + (-2 - iradius) * step) & ~3;
            const int W4 = (ix + (side + 1 - iradius) * step + 2 - cs + 3) >> 2;
            const int WP = 4 * W4;
            const int nitem = 2 * G * W4;
            const bool seg = step <= 3 && nitem <= 128 && 2 * G * WP <= 448;
            auto rows_seg = [&](auto AC) {
                constexpr bool A = decltype(AC)::value;
                uint32_t* buf = s_seg[w];
                // chunk i of a wave step: integral row rr = 2 g + e of the step's
                // grid rows, 16-byte chunk q; fixed per lane
                int ckoff[2], cdst[2];
                bool cok[2];
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    const int k = lane + 64 * i;
                    const int rr = k / W4, q = k - rr * W4;
                    cok[i] = k < nitem;
                    cdst[i] = rr * WP + 4 * q;
                    // integral row of grid row t0 (+ g): iy + (t0 + g - iradius) step + e
                    ckoff[i] = ((iy + (t0 + (rr >> 1) - iradius) * step + (rr & 1)) * P.ip + cs + 4 * q) * 4;
                }
                const int gstride = 2 * step * ip4;             // two grid rows further down
                struct Seg { uint4 c0, c1; };
                auto ldseg = [&](int tt) {                      // grid rows t0 + tt (+ 1): tt relative
                    Seg q;
                    const int d = tt * step * ip4;
                    q.c0 = buf_ld4(rsrc, cok[0] ? (uint32_t)(ckoff[0] + d) : kOOB);
                    q.c1 = buf_ld4(rsrc, cok[1] ? (uint32_t)(ckoff[1] + d) : kOOB);
                    return q;
                };
                const int xo = ld_on ? c - cs : 2 * hs;         // this lane's column in the buffer
                const int rowg = (dual ? h : 0) * 2 * WP;
                // T = rows r, r+1 x cols c-s, c, c+1, c+s+1
                auto proc = [&](const Seg& q, uint32_t (&T)[8]) {
                    if (cok[0]) *reinterpret_cast<uint4*>(buf + cdst[0]) = q.c0;
                    if (cok[1]) *reinterpret_cast<uint4*>(buf + cdst[1]) = q.c1;
                    lds_order();
                    const uint32_t* r0 = buf + rowg + xo;
                    const uint32_t* r1 = r0 + WP;
                    T[0] = r0[-hs]; T[1] = r0[0]; T[2] = r0[1]; T[3] = r0[hs + 1];
                    T[4] = r1[-hs]; T[5] = r1[0]; T[6] = r1[1]; T[7] = r1[hs + 1];
                    lds_order();
                };
                (void)gstride;
                for (int ph = 0; ph < (dual ? 1 : 2); ph++) {
                    const int hh = dual ? h : ph;
                    const int nstep = max(nv - hh + 1, 0) >> 1;
                    const int nmax = dual ? max(nv + 1, 0) >> 1 : nstep;
                    if (nmax == 0) continue;
                    // grid-row offset of this phase's first row relative to t0
                    // (dual: the chunks carry both halves' rows)
                    const int pb = dual ? 0 : ph;
                    auto sample = [&](int n, const uint32_t (&Pv)[8], const uint32_t (&Cv)[8],
                                      const uint32_t (&Nv)[8]) {
                        const int t = t0 + hh + 2 * n;
                        if (!(col_on && n < nstep)) return;
                        constexpr bool ok = true;
#ifdef SURF_DIAG_NOCOMP
                        acc[0][0] += (float)(Pv[0] ^ Cv[3] ^ Nv[5] ^ Pv[7] ^ Nv[1]);
                        return;
#endif
                        const float rp = s_rp[w][t];
                        const float4 wr = s_wr[w][t];
                        const uint32_t a00 = A ? Pv[0] : Pv[4], a02 = A ? Pv[1] : Pv[5];
                        const uint32_t a03 = A ? Pv[2] : Pv[6], a01 = A ? Pv[3] : Pv[7];
                        const uint32_t a30 = A ? Nv[4] : Nv[0], a32 = A ? Nv[5] : Nv[1];
                        const uint32_t a33 = A ? Nv[6] : Nv[2], a31 = A ? Nv[7] : Nv[3];
                        const uint32_t a10 = Cv[0], a11 = Cv[3], a20 = Cv[4], a21 = Cv[7];
                        const int32_t wav1 = (int32_t)((a21 + a00 - a01 - a20) - (a31 + a10 - a11 - a30));
                        const int32_t wav2 = (int32_t)((a31 + a02 - a01 - a32) - (a33 + a00 - a03 - a30));
                        float S[NS];
                        haar_bins(wav1, wav2, s_lut[f2i_rz(rp + cp2)], ok, S);
                        const float wrr[WSZ] = {wr.x, wr.y, wr.z, wr.w};
#pragma unroll
                        for (int R = 0; R < WSZ; R++)
#pragma unroll
                            for (int e = 0; e < NS; e++) acc[R][e] = fmaf(S[e], wrr[R], acc[R][e]);
                    };
                    uint32_t X[8], Y[8], Z[8];
                    // all five row loads in flight before the first LDS
                    // staging (proc's fences would otherwise hold each load
                    // back until the previous rows are staged: three memory
                    // round trips per keypoint before the loop)
#ifndef SURF_DIAG_DESC_SERIAL
                    const Seg q0 = ldseg(pb - 2), q1 = ldseg(pb);
                    Seg s0 = ldseg(pb + 2), s1 = ldseg(pb + 4), s2 = ldseg(pb + 6);
                    proc(q0, X);
                    proc(q1, Y);
#else
                    const Seg q0 = ldseg(pb - 2);
                    proc(q0, X);
                    const Seg q1 = ldseg(pb);
                    proc(q1, Y);
                    Seg s0 = ldseg(pb + 2), s1 = ldseg(pb + 4), s2 = ldseg(pb + 6);
#endif
#ifdef SURF_DIAG_NOROWS
                    continue;
#endif
                    for (int n = 0; n < nmax; n += 3) {
                        const int tt = pb + 2 * n;
                        proc(s0, Z);
                        s0 = ldseg(tt + 8);
                        sample(n, X, Y, Z);
                        proc(s1, X);
                        s1 = ldseg(tt + 10);
                        sample(n + 1, Y, Z, X);
                        proc(s2, Y);
                        s2 = ldseg(tt + 12);
                        sample(n + 2, Z, X, Y);
                    }
                }
            };
            if (seg) {
                if (hmode == 0) rows_seg(std::integral_constant<bool, true>());
                else rows_seg(std::integral_constant<bool, false>());
            } else {
                if (hmode == 0) rows(std::integral_constant<bool, true>());
                else rows(std::integral_constant<bool, false>());
            }
        } else {
            // ---- generic (hs = 2 step + 1 at exact half-way scales): 12
            // gathers per sample
            for (int k = h; k < nv; k += rstep) {
                if (col_on) {
                    const int rb = (iy + (t0 + k - iradius) * step) * ip4;
                    const int q0 = rb + dR0, q2 = rb + ip4, q3 = rb + dR3;
                    accum(bld(rsrc, q0 + oA), bld(rsrc, q0 + oB), bld(rsrc, q0 + oC), bld(rsrc, q0 + oC + 4),
                          bld(rsrc, rb + oA), bld(rsrc, rb + oB), bld(rsrc, q2 + oA), bld(rsrc, q2 + oB),
                          bld(rsrc, q3 + oA), bld(rsrc, q3 + oB), bld(rsrc, q3 + oC), bld(rsrc, q3 + oC + 4),
                          t0 + k);
                }
            }
        }
        // ---- per-lane bins, then the fixed-order column reduction
#pragma unroll
        for (int R = 0; R < WSZ; R++)
#pragma unroll
            for (int q = 0; q < NB / 2; q++) {
                red[w][lane][R * NB + 2 * q] = acc[R][2 * q + 1];                    // negative part
                red[w][lane][R * NB + 2 * q + 1] = acc[R][2 * q] - acc[R][2 * q + 1];
            }
        s_cf[w][lane] = cfrac;
        // The lanes of one cell column (ci == C) are one contiguous run per
        // half (cx and the image-bounds test are monotonic in j); the run's
        // [lo, hi) per half goes to s_run[C + 1] = {lo0, hi0, lo1, hi1}.
#pragma unroll
        for (int C = -1; C < WSZ; C++) {
            const unsigned long long mc = __ballot(col_on && ci == C);
            const uint32_t mlo = (uint32_t)mc, mhi = (uint32_t)(mc >> 32);
            if (lane == 0)
                s_run[w][C + 1] = make_int4(mlo ? __builtin_ctz(mlo) : 0, mlo ? 32 - __builtin_clz(mlo) : 0,
                                            mhi ? 32 + __builtin_ctz(mhi) : 32, mhi ? 64 - __builtin_clz(mhi) : 32);
        }
        wave_sync();
        float v[NF / 64];
#pragma unroll
        for (int hh = 0; hh < NF / 64; hh++) {
            const int o = lane + 64 * hh;                 // (R * WSZ + C) * NB + b
            const int b = o % NB, C = (o / NB) % WSZ, R = o / (NB * WSZ);
            const int col = R * NB + b;
            float s = 0.f;
            // cell column C: its own lanes at weight 1 - cfrac, then the lanes
            // of column C - 1 at cfrac; ascending lanes, 4 reads in flight
            auto run = [&](int lo, int hi, bool own) {
                int k = lo;
                for (; k + 4 <= hi; k += 4) {
                    float r[4], c[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) { r[u] = red[w][k + u][col]; c[u] = s_cf[w][k + u]; }
#pragma unroll
                    for (int u = 0; u < 4; u++) s += r[u] * (own ? 1.f - c[u] : c[u]);
                }
                for (; k < hi; k++) {
                    const float c = s_cf[w][k];
                    s += red[w][k][col] * (own ? 1.f - c : c);
                }
            };
#ifndef SURF_DIAG_NORED
            const int4 q0 = s_run[w][C + 1], q1 = s_run[w][C];
            run(q0.x, q0.y, true);
            run(q0.z, q0.w, true);
            run(q1.x, q1.y, false);
            run(q1.z, q1.w, false);
#else
            s = red[w][lane][col];
#endif
            v[hh] = s;
        }
        wave_sync();
        // ---- normalize (surfd.cu:2447-2493): sequential-addressing tree
        float a = v[0] * v[0];
        if constexpr (NF > 64) a = a + v[NF / 64 - 1] * v[NF / 64 - 1];
#pragma unroll
        for (int k = 32; k >= 1; k >>= 1) a = a + __shfl_down(a, k, 64);
        const float fac = 1.f / sqrtf(__shfl(a, 0, 64));
        float* out = desc + ((size_t)f * max_pts + kp) * NF;
        out[lane] = v[0] * fac;
        if constexpr (NF > 64) out[lane + 64] = v[NF / 64 - 1] * fac;
    }
}

#include "surfhip_desc_u2.inc"

// The describe schedule flattened for k_describe_u2: entry offsets[f] + i =
// keypoint order[f][i]'s {x, y, scale, f * max_pts + kp}, so the describe
// loop reaches a keypoint in one load after its queue atomic (order[] and
// pts[] were two dependent loads, and the frame a search over offsets[]).
__global__ __launch_bounds__(256) void k_worklist(const surfhip_point* __restrict__ pts, int max_pts,
                                                  const int* __restrict__ counts, const int* __restrict__ offsets,
                                                  const int* __restrict__ order, float4* __restrict__ work,
                                                  FrameParams P)
{
    // a frame's entries over gridDim.x workgroups, strided (most of a
    // max_pts-sized grid would find nothing to do).  Entry = three float4:
    // the keypoint's window geometry, the describe kernel's per-keypoint
    // set-up moved here (surfd.cu:1581-1596, the upright branch of describe),
    // then the point's laplace / ori words (getTrace's inputs when the fit
    // left it to the describe, nms_fit_point):
    //   {dx, dy, spacing, f}  {ix, iy, step | hs << 10 | iradius << 22, f * max_pts + kp}
    //   {laplace, ori, 1 / spacing, 0}
    // (10 / 12 / 10 bits: launch_describe takes this path only when the
    // largest window of the detector's octaves fits, worklist_fits)
    const int f = blockIdx.y, n = counts[f], o = offsets[f];
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int idx = f * max_pts + order[(size_t)f * max_pts + i];
        const surfhip_point p = pts[idx];
        const DescAt at = desc_at(P.doubled, p);
        const float scale = at.scale;
        const int step = max(f2i_rn(scale * 0.5f), 1);
#ifdef SURF_DIAG_WL_SAMEPOS
        // (diagnostic: every window of a frame at the frame's centre -- its
        // rows stay in L2; wrong descriptors, the same work)
        const int ix = P.W / 2, iy = P.H / 2;
#else
        const int ix = f2i_rn(at.x), iy = f2i_rn(at.y);
#endif
        const float spacing = scale * (float)P.mag;
        const int hs = f2i_rz(scale);
        const int iradius = f2i_rn(((spacing * (float)(P.wsz + 1)) * 0.5f) / (float)step);
        float4* e = work + kWorkF4 * (size_t)(o + i);
        e[0] = make_float4(at.x - (float)ix, at.y - (float)iy, spacing, __int_as_float(f));
        e[1] = make_float4(__int_as_float(ix), __int_as_float(iy), __int_as_float(step | (hs << 10) | (iradius << 22)),
                           __int_as_float(idx));
        e[2] = make_float4(__int_as_float(p.laplace), p.ori, 1.f / spacing, 0.f);
    }
}

// Whether k_worklist's packed fields hold every keypoint window of this
// detector: the largest keypoint scale is makePoint's 1.2 ns
// divisor (surfd.cu:1001-1022) at the top octave with s + off <= max_scale -
// 1 + 1.5 (the fit's limits); describe uses 1.65 x (3.3 x doubled) of it
// (surfd.cu:1581-1592); step = rn(S / 2) < 2^10, hs = rz(S) < 2^12, iradius
// = rn(spacing (wsz + 1) / 2 / step) < 2^10.
static bool worklist_fits(const FrameParams& P)
{
    const float oct = (float)(1 << (P.noct - 1));
    const float ns = ((float)P.init_lobe + (oct - 1.f) * (float)P.max_scale + ((float)P.max_scale + 0.5f) * 2.f * oct) / 3.f;
    const float S = (P.doubled ? 3.3f : 1.65f) * 1.2f * ns * P.divisor;
    const float step = std::max(std::floor(S * 0.5f + 0.5f), 1.f);
    const float iradius = S * (float)P.mag * (float)(P.wsz + 1) * 0.5f / step + 1.f;
    return S * 0.5f + 1.f < 1024.f && S + 1.f < 4096.f && iradius < 1024.f;
}

bool describe_on_u2(const FrameParams& P, int nframes)
{
    // SURFHIP_DESC_UR=1 / 0 forces k_describe_ur / k_describe_u2 (read per
    // call, so a process can A/B both kernels); default: k_describe_ur for
    // batches of <= kGatherBatch frames, where a wave gets about one keypoint
    // and the ring's fill latency is not amortised -- one 1080p frame's
    // describe 0.032 -> 0.030 ms
    const char* ur = getenv("SURFHIP_DESC_UR");
    const bool use_u2 = ur ? atoi(ur) == 0 : nframes > kGatherBatch;
    return P.upright && P.wsz == 4 && use_u2 && worklist_fits(P);
}

bool trace_in_describe(const FrameParams& P, int nframes)
{
    const char* e = getenv("SURFHIP_TRACE_DESC");
    return (e ? atoi(e) != 0 : true) && describe_on_u2(P, nframes);
}

hipError_t launch_describe(const int32_t* ii, const FrameParams& P, surfhip_point* pts, int max_pts,
                           const int* counts, const int* offsets, const int* order, float4* work, int nframes,
                           float* desc, int* queue, hipStream_t s, bool beside, int cus, bool trace)
{
    if (P.nfeat > 512) return hipErrorInvalidValue;
    // the describe kernels are persistent (per-XCD keypoint queues): 2,048
    // workgroups fill every CU; with another stream's kernels beside them
    // (SURFHIP_DESC_BESIDE workgroups per CU, default 3) a slot stays free
    if (cus <= 0) cus = 256;
    static const int per_cu = getenv("SURFHIP_DESC_BESIDE") ? atoi(getenv("SURFHIP_DESC_BESIDE")) : 3;
    const int grid = (beside && per_cu > 0) ? ((per_cu * cus + 7) & ~7) : 2048;
    hipError_t e = hipMemsetAsync(queue, 0, kDescQueueBytes, s);
    if (e != hipSuccess) return e;
    // k_describe_u2 (LDS-DMA ring), else round 3's k_describe_ur
    // (describe_on_u2); `trace` implies the u2 path (trace_in_describe)
    const bool u2 = describe_on_u2(P, nframes);
    if (trace && !u2) return hipErrorInvalidValue;
    if (u2) {
        k_worklist<<<dim3(std::min(8, (max_pts + 255) / 256), nframes), 256, 0, s>>>(pts, max_pts, counts, offsets,
                                                                                      order, work, P);
        // (diagnostic: SURFHIP_U2_LDSPAD bytes of unused dynamic LDS per workgroup)
        static const int pad = getenv("SURFHIP_U2_LDSPAD") ? atoi(getenv("SURFHIP_U2_LDSPAD")) : 0;
        const int tr = trace ? 1 : 0;
        if (P.extend)
            k_describe_u2<true><<<grid, 256, pad, s>>>(ii, P, work, max_pts, offsets, nframes, desc, queue, pts, tr);
        else k_describe_u2<false><<<grid, 256, pad, s>>>(ii, P, work, max_pts, offsets, nframes, desc, queue, pts, tr);
    } else if (P.upright && P.wsz == 4) {
        if (P.extend)
            k_describe_ur<true><<<grid, 256, 0, s>>>(ii, P, pts, max_pts, offsets, order, nframes, desc, queue);
        else k_describe_ur<false><<<grid, 256, 0, s>>>(ii, P, pts, max_pts, offsets, order, nframes, desc, queue);
    } else if (P.nfeat > 128) {
        // windows past 4 x 4 x 8 (desc_wsz 5..7: up to 392 features)
        if (P.upright)
            k_describe<true, 512><<<grid, 256, 0, s>>>(ii, P, pts, max_pts, counts, offsets, order, nframes, desc, queue);
        else
            k_describe<false, 512><<<grid, 256, 0, s>>>(ii, P, pts, max_pts, counts, offsets, order, nframes, desc, queue);
    } else if (P.upright) {
        k_describe<true, 128><<<grid, 256, 0, s>>>(ii, P, pts, max_pts, counts, offsets, order, nframes, desc, queue);
    } else if (P.wsz == 4 && getenv("SURFHIP_ROT_ATOMIC") == nullptr) {
        if (P.osz == 8)
            k_describe_rot<8><<<grid, 256, 0, s>>>(ii, P, pts, max_pts, offsets, order, nframes, desc, queue);
        else k_describe_rot<4><<<grid, 256, 0, s>>>(ii, P, pts, max_pts, offsets, order, nframes, desc, queue);
    } else {
        k_describe<false, 128><<<grid, 256, 0, s>>>(ii, P, pts, max_pts, counts, offsets, order, nframes, desc, queue);
    }
    return hipGetLastError();
}

// ======================================================================
// Result slab for the multi-GPU all-gather, compacted:
//   int32 header[4] = {nframes, total, nfeatures, 0}
//   int32 counts[nframes] (padded to 16 B)
//   SurfPoint points[total]            frame-major, canonical order
//   float     desc[total][nfeatures]   (absent when desc == nullptr)
// offsets[] is the exclusive prefix of counts written by k_offsets.
// ======================================================================
__global__ __launch_bounds__(256) void k_pack(const surfhip_point* __restrict__ pts, const float* __restrict__ desc,
                                              const int* __restrict__ counts, const int* __restrict__ offsets,
                                              int nframes, int max_pts, int nfeat, const int* __restrict__ status,
                                              size_t cap_bytes, uint8_t* __restrict__ slab)
{
    const int f = blockIdx.y;
    const int total = offsets[nframes];
    const size_t head = 16 + (((size_t)nframes * 4 + 15) & ~(size_t)15);
    const size_t need = head + (size_t)total * (sizeof(surfhip_point) + (desc ? 4 * (size_t)nfeat : 0));
    const bool fits = need <= cap_bytes;
    int* hdr = reinterpret_cast<int*>(slab);
    if (f == 0 && blockIdx.x == 0) {
        // hdr[3] bit 0: a frame of this batch was truncated at the candidate
        // capacity; bit 1: the slab did not fit cap_bytes (payload not written)
        if (threadIdx.x == 0) {
            hdr[0] = nframes;
            hdr[1] = total;
            hdr[2] = desc ? nfeat : 0;
            hdr[3] = (status ? (*status & 1) : 0) | (fits ? 0 : 2);
        }
        const int npad = (nframes + 3) & ~3;          // counts padded to 16 B with zeros (stable file bytes)
        for (int i = threadIdx.x; i < npad; i += 256) hdr[4 + i] = i < nframes ? counts[i] : 0;
    }
    if (!fits) return;
    surfhip_point* pout = reinterpret_cast<surfhip_point*>(slab + head);
    float* dout = reinterpret_cast<float*>(slab + head + (size_t)total * sizeof(surfhip_point));
    const int cnt = counts[f], off = offsets[f];
    const size_t tid = (size_t)blockIdx.x * 256 + threadIdx.x, stride = (size_t)gridDim.x * 256;
    for (size_t t = tid; t < (size_t)cnt; t += stride) pout[off + t] = pts[(size_t)f * max_pts + t];
    if (desc) {
        const float* src = desc + (size_t)f * max_pts * nfeat;
        float* dst = dout + (size_t)off * nfeat;
        const size_t n4 = (size_t)cnt * nfeat / 4;          // nfeat is 64 or 128
        for (size_t t = tid; t < n4; t += stride)
            reinterpret_cast<float4*>(dst)[t] = reinterpret_cast<const float4*>(src)[t];
    }
}

hipError_t launch_pack(const surfhip_point* pts, const float* desc, const int* counts, const int* offsets,
                       int nframes, int max_pts, int nfeat, const int* status, size_t cap_bytes, uint8_t* slab,
                       hipStream_t s)
{
    k_pack<<<dim3(16, nframes), 256, 0, s>>>(pts, desc, counts, offsets, nframes, max_pts, nfeat, status,
                                             cap_bytes, slab);
    return hipGetLastError();
}

#ifdef SURF_DIAG_U2_STAMP
extern "C" int surfhip_diag_u2_stamps(unsigned long long* host)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dstamp), sizeof(g_dstamp)) == hipSuccess ? 0 : -1;
}
#endif
#ifdef SURF_DIAG_W_STAMP
extern "C" int surfhip_diag_w_stamps(unsigned long long* host)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wstamp), sizeof(g_wstamp)) == hipSuccess ? 0 : -1;
}
#endif

}  // namespace surfhip
