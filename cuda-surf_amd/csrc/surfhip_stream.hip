// surfhip_stream.hip -- the measured HBM stream rates the roofline is also
// priced against ("Also report measured peak from an in-repo
// stream-copy kernel").  No reference counterpart: the
// reference never measures bandwidth.
//
// One 16-B load and/or store per lane per step, 4 steps unrolled so each
// lane keeps 4 loads in flight, grid-stride over the buffer; the grid is 8
// workgroups of 256 per CU (one launch fills the chip several times over).
// Copy and read use non-temporal loads (each byte is read once), stores
// the default policy (measured faster for the plane / integral writers,
// DESIGN §4).  The read kernel keeps its sums live by a store that never
// happens for real data (an XOR equal to a 64-bit magic).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "surfhip_internal.h"

namespace surfhip {

namespace {

constexpr int kStreamUnroll = 4;
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_stream_copy(const u4* __restrict__ src, u4* __restrict__ dst, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (kStreamUnroll - 1) * stride < n; i += kStreamUnroll * stride) {
        u4 v[kStreamUnroll];
#pragma unroll
        for (int k = 0; k < kStreamUnroll; k++) v[k] = __builtin_nontemporal_load(src + i + k * stride);
#pragma unroll
        for (int k = 0; k < kStreamUnroll; k++) dst[i + k * stride] = v[k];
    }
    for (; i < n; i += stride) dst[i] = __builtin_nontemporal_load(src + i);
}

__global__ __launch_bounds__(256) void k_stream_read(const u4* __restrict__ src, u4* __restrict__ dst, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t a = 0u, b = 0u;
    for (; i + (kStreamUnroll - 1) * stride < n; i += kStreamUnroll * stride) {
        u4 v[kStreamUnroll];
#pragma unroll
        for (int k = 0; k < kStreamUnroll; k++) v[k] = __builtin_nontemporal_load(src + i + k * stride);
#pragma unroll
        for (int k = 0; k < kStreamUnroll; k++) {
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

__global__ __launch_bounds__(256) void k_stream_write(u4* __restrict__ dst, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const u4 v = {(uint32_t)i, 1u, 2u, 3u};
    for (; i < n; i += stride) dst[i] = v;
}

}  // namespace

hipError_t launch_stream(int mode, const void* src, void* dst, size_t bytes, int ncu, hipStream_t s)
{
    const size_t n = bytes / 16;
    const dim3 grid((unsigned)(8 * (ncu > 0 ? ncu : 256)));
    if (mode == 0)
        k_stream_copy<<<grid, 256, 0, s>>>((const u4*)src, (u4*)dst, n);
    else if (mode == 1)
        k_stream_read<<<grid, 256, 0, s>>>((const u4*)src, (u4*)dst, n);
    else
        k_stream_write<<<grid, 256, 0, s>>>((u4*)dst, n);
    return hipGetLastError();
}

}  // namespace surfhip
