// surfhip_stream.hip -- the measured HBM stream rates the roofline is also
// priced against ("Also report measured peak from an in-repo
// stream-copy kernel").  No reference counterpart: the
// reference never measures bandwidth.
//
// 16-B accesses per lane, several in flight.  The read kernel keeps its
// sums live by a store that never happens for real data (an XOR equal to a
// 64-bit magic).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "surfhip_internal.h"

namespace surfhip {

namespace {

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

// The forms below are the fastest of tools/ubench/stream_sweep.hip's sweep
// (profiles/r06b/stream_sweep.txt, 2-GiB buffers): copy as contiguous
// per-workgroup chunks with non-temporal loads and stores, 8 workgroups per
// CU (5.36 TB/s read + write; grid-stride forms 4.1-4.96); read grid-stride
// with 8 non-temporal 16-B loads in flight per lane, 32 workgroups per CU
// (6.24 TB/s); write grid-stride, 4 default-policy 16-B stores per lane, 8
// workgroups per CU (4.64 TB/s; nt stores 4.42-4.45).
constexpr int kCopyU = 4;

__global__ __launch_bounds__(256) void k_stream_copy(const u4* __restrict__ src, u4* __restrict__ dst, size_t n,
                                                     size_t per_wg)
{
    const size_t b0 = (size_t)blockIdx.x * per_wg;
    const size_t e = b0 + per_wg < n ? b0 + per_wg : n;
    for (size_t i = b0 + threadIdx.x; i < e; i += kCopyU * 256) {
        u4 v[kCopyU];
#pragma unroll
        for (int k = 0; k < kCopyU; k++)
            v[k] = i + k * 256 < e ? __builtin_nontemporal_load(src + i + k * 256) : u4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < kCopyU; k++)
            if (i + k * 256 < e) __builtin_nontemporal_store(v[k], dst + i + k * 256);
    }
}

constexpr int kReadU = 8;

__global__ __launch_bounds__(256) void k_stream_read(const u4* __restrict__ src, u4* __restrict__ dst, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t a = 0u, b = 0u;
    for (; i + (kReadU - 1) * stride < n; i += kReadU * stride) {
        u4 v[kReadU];
#pragma unroll
        for (int k = 0; k < kReadU; k++) v[k] = __builtin_nontemporal_load(src + i + k * stride);
#pragma unroll
        for (int k = 0; k < kReadU; k++) {
            a ^= v[k].x ^ v[k].z;
            b ^= v[k].y ^ v[k].w;
        }
    }
    for (; i < n; i += stride) {
        const u4 v = __builtin_nontemporal_load(src + i);
        a ^= v.x ^ v.z;
        b ^= v.y ^ v.w;
    }
    if (a == 0x9E3779B9u && b == 0x7F4A7C15u) dst[0] = u4{a, b, a, b};
}

constexpr int kWriteU = 4;

__global__ __launch_bounds__(256) void k_stream_write(u4* __restrict__ dst, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const u4 v = {(uint32_t)i, 1u, 2u, 3u};
    for (; i + (kWriteU - 1) * stride < n; i += kWriteU * stride) {
#pragma unroll
        for (int k = 0; k < kWriteU; k++) dst[i + k * stride] = v;
    }
    for (; i < n; i += stride) dst[i] = v;
}

}  // namespace

hipError_t launch_stream(int mode, const void* src, void* dst, size_t bytes, int ncu, hipStream_t s)
{
    const size_t n = bytes / 16;
    if (ncu <= 0) ncu = 256;
    if (mode == 0) {
        const unsigned g = (unsigned)(8 * ncu);
        k_stream_copy<<<g, 256, 0, s>>>((const u4*)src, (u4*)dst, n, (n + g - 1) / g);
    } else if (mode == 1) {
        k_stream_read<<<(unsigned)(32 * ncu), 256, 0, s>>>((const u4*)src, (u4*)dst, n);
    } else {
        k_stream_write<<<(unsigned)(8 * ncu), 256, 0, s>>>((u4*)dst, n);
    }
    return hipGetLastError();
}

}  // namespace surfhip
