// surfhip_double.hip -- the doubled-image input (SurfParam.doubled = true).
//
// Reference: cuIntegralDoubleU4 (surfd.cu:2707-2772) with its six kernels
// integralDoubleRow0U2 / integralRow1U4 / integralRow2U4 / integralCol0U4 /
// integralCol1U4 / integralCol2U4 (surfd.cu:166-318): the integral image,
// on the (2W-1) x (2H-1) grid of surf.cpp:377-378, of the 2x upsampled frame
//   D[2y][2x]     = s[y][x]
//   D[2y][2x+1]   = rn((s[y][x] + s[y][x+1]) * 0.5f)
//   D[2y+1][2x]   = rn((s[y][x] + s[y+1][x]) * 0.5f)
//   D[2y+1][2x+1] = rn((s[y][x] + s[y][x+1] + s[y+1][x] + s[y+1][x+1]) * 0.25f)
// (pinned against a literal run of the six kernels in tests/test_oracle.py).
// D is (2W-2) x (2H-2) u8 -- every value is a rounded mean of u8 pixels -- so
// the engine materialises D once per frame (k_double, one pass, 4 output
// bytes per thread) and runs its ordinary integral-image and Hessian kernels
// on it: no separate scan, and the integral stays exact.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "surfhip_internal.h"

namespace surfhip {

namespace {

__global__ __launch_bounds__(256) void k_double(const uint8_t* __restrict__ src, int pitch, long long fstride,
                                                int W, int H, uint8_t* __restrict__ dst, int dpitch,
                                                long long dstride)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;    // D columns 4t .. 4t + 3
    const int r = blockIdx.y, f = blockIdx.z;
    const int c0 = 4 * t;
    if (c0 >= dpitch) return;
    const int W2 = 2 * W - 2;
    const int y = r >> 1;
    const uint8_t* s0 = src + (size_t)f * fstride + (size_t)y * pitch;
    const uint8_t* s1 = (r & 1) ? s0 + pitch : s0;           // row y + 1 only for odd D rows (y + 1 < H)
    const int x0 = c0 >> 1;                                  // source columns x0, x0 + 1, x0 + 2
    int a[3], b[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const int x = x0 + k;
        a[k] = x < W ? (int)s0[x] : 0;
        b[k] = x < W ? (int)s1[x] : 0;
    }
    uint32_t out = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int c = c0 + k;
        const int i = k >> 1;                                // x = x0 + i
        int v;
        if (!(r & 1) && !(k & 1)) v = a[i];
        else if (!(r & 1)) v = __float2int_rn((float)(a[i] + a[i + 1]) * 0.5f);
        else if (!(k & 1)) v = __float2int_rn((float)(a[i] + b[i]) * 0.5f);
        else v = __float2int_rn((float)(a[i] + a[i + 1] + b[i] + b[i + 1]) * 0.25f);
        if (c >= W2) v = 0;
        out |= (uint32_t)v << (8 * k);
    }
    *reinterpret_cast<uint32_t*>(dst + (size_t)f * dstride + (size_t)r * dpitch + c0) = out;
}

}  // namespace

hipError_t launch_double(const uint8_t* frames, int pitch, long long fstride, int nframes, int W, int H,
                         uint8_t* dst, int dpitch, long long dstride, hipStream_t s)
{
    const int H2 = 2 * H - 2;
    const dim3 grid((dpitch / 4 + 255) / 256, H2, nframes);
    k_double<<<grid, 256, 0, s>>>(frames, pitch, fstride, W, H, dst, dpitch, dstride);
    return hipGetLastError();
}

}  // namespace surfhip
