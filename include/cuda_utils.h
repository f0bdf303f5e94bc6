// cuda_utils.h -- thin layer over the libsurfhip C-ABI that keeps the names
// the reference's callers use (CUDA-SURF cuda_utils.h:1-170 and the handful
// of runtime calls main.cpp:12-283 makes through it).
//
// No CUDA or HIP headers are included: every call below is one surfhip_*
// entry point of include/surfhip.h.  Error handling keeps the reference
// convention (print file/line and exit(-1), cuda_utils.h:18-37).
#pragma once

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>

#include "surfhip.h"

#define H_PI 1.5707963267948966f

// ---- vector type used in the public API (surf.h detectAndCompute's whp0)
struct int3
{
    int x, y, z;
};
static_assert(sizeof(int3) == 12, "int3 must be 12 bytes");

// ---- status type of the wrapped runtime calls
typedef int cudaError;
typedef int cudaError_t;
static const int cudaSuccess = SURFHIP_OK;
enum cudaMemcpyKind
{
    cudaMemcpyHostToHost = SURFHIP_H2H,
    cudaMemcpyHostToDevice = SURFHIP_H2D,
    cudaMemcpyDeviceToHost = SURFHIP_D2H,
    cudaMemcpyDeviceToDevice = SURFHIP_D2D
};
typedef void* cudaStream_t;

inline const char* cudaGetErrorString(int err) { return surfhip_error_string(err); }

#define CHECK(err) __check(err, __FILE__, __LINE__)
#define CheckMsg(msg) __checkMsg(msg, __FILE__, __LINE__)

inline void __check(int err, const char* file, const int line)
{
    if (err != SURFHIP_OK)
    {
        fprintf(stderr, "CHECK() Runtime API error in file <%s>, line %i : %s.\n", file, line,
                surfhip_error_string(err));
        exit(-1);
    }
}

// Launch errors are reported synchronously by the C-ABI, so there is no
// deferred error to poll; kept for source compatibility.
inline void __checkMsg(const char* msg, const char* file, const int line)
{
    (void)msg;
    (void)file;
    (void)line;
}

// ---- runtime calls used by main.cpp
template <class T>
inline int cudaMalloc(T** ptr, size_t bytes) { return surfhip_malloc(reinterpret_cast<void**>(ptr), bytes); }
template <class T>
inline int cudaMallocPitch(T** ptr, size_t* pitch, size_t width_bytes, size_t height)
{
    return surfhip_malloc_pitch(reinterpret_cast<void**>(ptr), pitch, width_bytes, height);
}
inline int cudaFree(void* ptr) { return surfhip_free(ptr); }
inline int cudaMemset(void* ptr, int v, size_t n) { return surfhip_memset(ptr, v, n); }
inline int cudaMemcpy(void* dst, const void* src, size_t n, cudaMemcpyKind k) { return surfhip_memcpy(dst, src, n, k); }
inline int cudaMemcpy2D(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t height,
                        cudaMemcpyKind k)
{
    return surfhip_memcpy2d(dst, dpitch, src, spitch, width, height, k);
}
inline int cudaDeviceSynchronize() { return surfhip_device_synchronize(); }
inline int cudaDeviceReset() { return surfhip_device_reset(); }

// ---- initDevice (cuda_utils.h:41-67)
inline bool initDevice(int dev)
{
    int count = 0;
    CHECK(surfhip_get_device_count(&count));
    if (count == 0)
    {
        fprintf(stderr, "HIP error: no devices.\n");
        return false;
    }
    dev = std::max<int>(0, std::min<int>(dev, count - 1));
    CHECK(surfhip_set_device(dev));
    char name[256];
    int cus = 0, drv = 0, rt = 0;
    CHECK(surfhip_device_name(dev, name, sizeof(name), &cus));
    CHECK(surfhip_versions(&drv, &rt));
    fprintf(stderr, "Using Device %d: %s, %d CUs, HIP Driver Version: %d, Runtime Version: %d\n", dev, name, cus,
            drv, rt);
    return true;
}

// ---- cpuTimer (cuda_utils.h:71-77): microseconds since the epoch
inline long long cpuTimer()
{
    return std::chrono::duration_cast<std::chrono::microseconds>(
               std::chrono::system_clock::now().time_since_epoch())
        .count();
}

// ---- GpuTimer (cuda_utils.h:81-108): ms since construction, on a stream
class GpuTimer
{
public:
    GpuTimer(cudaStream_t stream_ = 0) : stream(stream_)
    {
        surfhip_event_create(&start);
        surfhip_event_create(&stop);
        surfhip_event_record(start, stream);
    }
    ~GpuTimer()
    {
        surfhip_event_destroy(start);
        surfhip_event_destroy(stop);
    }
    float read()
    {
        float ms = 0.f;
        surfhip_event_record(stop, stream);
        surfhip_event_synchronize(stop);
        surfhip_event_elapsed(&ms, start, stop);
        return ms;
    }

private:
    void* start = nullptr;
    void* stop = nullptr;
    cudaStream_t stream;
};

// ---- iAlignUp / iDivUp (cuda_utils.h:160-170)
inline int iAlignUp(const int a, const int b) { return (a % b != 0) ? (a - a % b + b) : a; }
inline int iDivUp(int a, int b) { return (a % b != 0) ? (a / b + 1) : (a / b); }
