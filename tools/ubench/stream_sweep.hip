// stream_sweep.hip -- which form of a streaming HBM copy / read / write
// kernel reaches the highest rate on gfx950 (picks the form of the product's
// surfhip_stream_run, cuda-surf_amd/csrc/surfhip_stream.hip).  2-GiB buffers
// (8x the memory-side cache), 10 timed launches per variant.
//
//   hipcc --offload-arch=gfx950 -O3 -o stream_sweep stream_sweep.hip && ./stream_sweep
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

// LNT: non-temporal loads; SNT: non-temporal stores; U: 16-B accesses in flight per lane
template <int U, bool LNT, bool SNT>
__global__ __launch_bounds__(256) void k_copy(const u4* __restrict__ src, u4* __restrict__ dst, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        u4 v[U];
#pragma unroll
        for (int k = 0; k < U; k++) v[k] = LNT ? __builtin_nontemporal_load(src + i + k * stride) : src[i + k * stride];
#pragma unroll
        for (int k = 0; k < U; k++) {
            if (SNT) __builtin_nontemporal_store(v[k], dst + i + k * stride);
            else dst[i + k * stride] = v[k];
        }
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

// contiguous chunks per workgroup instead of grid-stride: a workgroup walks
// CH consecutive 4-KiB pieces
template <int U, bool SNT>
__global__ __launch_bounds__(256) void k_copy_chunk(const u4* __restrict__ src, u4* __restrict__ dst, size_t n,
                                                    size_t per_wg)
{
    const size_t b0 = (size_t)blockIdx.x * per_wg;
    const size_t e = b0 + per_wg < n ? b0 + per_wg : n;
    for (size_t i = b0 + threadIdx.x; i < e; i += U * 256) {
        u4 v[U];
#pragma unroll
        for (int k = 0; k < U; k++) v[k] = i + k * 256 < e ? __builtin_nontemporal_load(src + i + k * 256) : u4{0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < U; k++)
            if (i + k * 256 < e) {
                if (SNT) __builtin_nontemporal_store(v[k], dst + i + k * 256);
                else dst[i + k * 256] = v[k];
            }
    }
}

template <int U, bool LNT>
__global__ __launch_bounds__(256) void k_read(const u4* __restrict__ src, u4* __restrict__ dst, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t a = 0;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        u4 v[U];
#pragma unroll
        for (int k = 0; k < U; k++) v[k] = LNT ? __builtin_nontemporal_load(src + i + k * stride) : src[i + k * stride];
#pragma unroll
        for (int k = 0; k < U; k++) a ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (a == 0x9E3779B9u) dst[0] = u4{a, a, a, a};
}

template <int U, bool SNT>
__global__ __launch_bounds__(256) void k_write(u4* __restrict__ dst, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const u4 v = {(uint32_t)i, 1u, 2u, 3u};
    for (; i + (U - 1) * stride < n; i += U * stride) {
#pragma unroll
        for (int k = 0; k < U; k++) {
            if (SNT) __builtin_nontemporal_store(v, dst + i + k * stride);
            else dst[i + k * stride] = v;
        }
    }
    for (; i < n; i += stride) dst[i] = v;
}

template <typename F>
static float timeit(F f)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();
    f();
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < 10; r++) f();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms / 10;
}

int main()
{
    const size_t bytes = 2ull << 30, n = bytes / 16;
    u4 *s, *d;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(s, 1, bytes));
    CK(hipMemset(d, 0, bytes));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int wgs[] = {4, 8, 16, 32};
#define COPY(U, L, S)                                                                                      \
    for (int w : wgs) {                                                                                    \
        const dim3 g(w * ncu);                                                                             \
        const float ms = timeit([&] { k_copy<U, L, S><<<g, 256>>>(s, d, n); });                            \
        printf("copy U=%d ldnt=%d stnt=%d wg/cu=%2d: %7.1f GB/s (r+w)\n", U, L, S, w, 2.0 * bytes / ms / 1e6); \
    }
    COPY(4, true, false) COPY(4, true, true) COPY(4, false, false) COPY(8, true, false) COPY(8, true, true)
    COPY(2, true, false) COPY(1, true, false)
    for (int w : {1, 2, 4, 8}) {
        const dim3 g(w * ncu);
        const size_t per = (n + g.x - 1) / g.x;
        float ms = timeit([&] { k_copy_chunk<4, false><<<g, 256>>>(s, d, n, per); });
        printf("copy chunked U=4 stnt=0 wg/cu=%d: %7.1f GB/s\n", w, 2.0 * bytes / ms / 1e6);
        ms = timeit([&] { k_copy_chunk<4, true><<<g, 256>>>(s, d, n, per); });
        printf("copy chunked U=4 stnt=1 wg/cu=%d: %7.1f GB/s\n", w, 2.0 * bytes / ms / 1e6);
    }
#define READ(U, L)                                                                                      \
    for (int w : wgs) {                                                                                 \
        const dim3 g(w * ncu);                                                                          \
        const float ms = timeit([&] { k_read<U, L><<<g, 256>>>(s, d, n); });                            \
        printf("read U=%d ldnt=%d wg/cu=%2d: %7.1f GB/s\n", U, L, w, 1.0 * bytes / ms / 1e6);           \
    }
    READ(4, true) READ(4, false) READ(8, true) READ(16, true)
#define WRITE(U, S)                                                                                     \
    for (int w : wgs) {                                                                                 \
        const dim3 g(w * ncu);                                                                          \
        const float ms = timeit([&] { k_write<U, S><<<g, 256>>>(d, n); });                              \
        printf("write U=%d stnt=%d wg/cu=%2d: %7.1f GB/s\n", U, S, w, 1.0 * bytes / ms / 1e6);          \
    }
    WRITE(1, false) WRITE(1, true) WRITE(4, false) WRITE(4, true)
    {
        const float ms = timeit([&] { (void)hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); });
        printf("hipMemcpyAsync D2D: %7.1f GB/s (r+w)\n", 2.0 * bytes / ms / 1e6);
    }
    CK(hipDeviceSynchronize());
    CK(hipFree(s));
    CK(hipFree(d));
    return 0;
}
