// surf.cpp -- the drop-in C++ host API (include/surf.h) over the libsurfhip
// C-ABI.  Mirrors the reference's surf.cpp:10-428 call for call:
//   initSurfData/freeSurfData     surf.cpp:10-36
//   Surfor::init                  surf.cpp:60-91
//   Surfor::detectAndCompute      surf.cpp:205-355
// The per-frame work (integral, Hessian, NMS, describe) runs as HIP kernels
// inside libsurfhip; this file only owns the detector handle and the host
// copies the reference API promises.
#include "surf.h"

#include <cstdlib>
#include <cstring>

namespace surf
{
    static_assert(sizeof(SurfParam) == sizeof(surfhip_param), "SurfParam ABI");
    static_assert(sizeof(SurfPoint) == sizeof(surfhip_point), "SurfPoint ABI");

    void initSurfData(SurfData& data, const int max_pts, const bool host, const bool dev)
    {
        data.num_pts = 0;
        data.max_pts = max_pts;
        const size_t bytes = sizeof(SurfPoint) * (size_t)max_pts;
        data.h_data = host ? (SurfPoint*)malloc(bytes) : nullptr;
        data.d_data = nullptr;
        if (dev)
            CHECK(surfhip_malloc((void**)&data.d_data, bytes));
    }

    void freeSurfData(SurfData& data)
    {
        if (data.d_data != nullptr)
            CHECK(surfhip_free(data.d_data));
        if (data.h_data != nullptr)
            free(data.h_data);
        data.d_data = nullptr;
        data.h_data = nullptr;
        data.num_pts = 0;
        data.max_pts = 0;
    }

    Surfor::Surfor() {}

    Surfor::~Surfor()
    {
        if (det)
            surfhip_detector_destroy(det);
    }

    void Surfor::init(const int _noctaves, const float _thresh, const bool _doubled, const int _init_mask_size,
                      const int _sampling_step, const bool _upright, const bool _extend, const int _desc_wsz,
                      const int _width, const int _height)
    {
        surfhip_param p;
        const int rc = surfhip_make_param(&p, _noctaves, _thresh, _doubled, _init_mask_size, _sampling_step,
                                          _upright, _extend, _desc_wsz);
        if (rc != SURFHIP_OK)
        {
            fprintf(stderr, "Surfor::init: unsupported parameters (%s)\n", surfhip_error_string(rc));
            exit(-1);
        }
        memcpy(&its, &p, sizeof(its));
        whp.x = _width;
        whp.y = _height;
        whp.z = _width > 0 ? iAlignUp(_width, 128) : -1;
        if (det)
        {
            surfhip_detector_destroy(det);
            det = nullptr;
        }
    }

    void Surfor::detectAndCompute(unsigned char* image, SurfData& result, int3 whp0, float** desc_addr,
                                  const bool desc)
    {
        // scratch is kept for the geometry of the last call (the reference keeps
        // it for the init geometry and re-allocates per call otherwise,
        // surf.cpp:222-231, 350-354)
        if (!det || det_w != whp0.x || det_h != whp0.y || det_pts < result.max_pts)
        {
            if (det)
                surfhip_detector_destroy(det);
            det = nullptr;
            surfhip_param p;
            memcpy(&p, &its, sizeof(p));
            CHECK(surfhip_detector_create(&det, &p, whp0.x, whp0.y, 1, result.max_pts, 0, nullptr));
            det_w = whp0.x;
            det_h = whp0.y;
            det_pts = result.max_pts;
            warned_trunc = false;
        }
        int n = 0;
        float* dptr = nullptr;
        CHECK(surfhip_detect(det, image, whp0.z, reinterpret_cast<surfhip_point*>(result.d_data), result.max_pts, &n,
                             desc ? &dptr : nullptr, desc ? 1 : 0));
        result.num_pts = n;
        if (desc && desc_addr)
            *desc_addr = dptr;
        // more NMS survivors than the detector's candidate capacity: the frame
        // kept the first ones in scan order (deterministic, include/surfhip.h);
        // the reference keeps an arbitrary subset and says nothing
        // (surfd.cu:822-831) -- say it once per detector
        int trunc = 0;
        CHECK(surfhip_detector_status(det, &trunc));
        if (trunc && !warned_trunc)
        {
            int cap = 0;
            CHECK(surfhip_detector_capacity(det, &cap));
            fprintf(stderr, "Surfor::detectAndCompute: a frame had more than %d scale-space maxima; the first %d "
                            "in scan order were interpolated (raise max_pts to keep all)\n", cap, cap);
            warned_trunc = true;
        }
        // surf.cpp:335-342: the first 6 fields (7 with rotated descriptors)
        if (result.h_data != nullptr && n > 0)
        {
            const size_t fields = (desc && !its.upright) ? 7 : 6;
            CHECK(surfhip_memcpy2d(&result.h_data[0].x, sizeof(SurfPoint), &result.d_data[0].x, sizeof(SurfPoint),
                                   fields * sizeof(float), (size_t)n, SURFHIP_D2H));
        }
    }

    void Surfor::match(SurfData& data1, SurfData& data2, float* features1, float* features2)
    {
        // surf.cpp:418-428: cuFindMaxCorr on the device (synchronous, as the
        // reference's cudaDeviceSynchronize), then score, match, match_x,
        // match_y, ambiguity (5 consecutive 4-B fields at offset 28) to h_data.
        CHECK(surfhip_match(reinterpret_cast<surfhip_point*>(data1.d_data),
                            reinterpret_cast<const surfhip_point*>(data2.d_data), features1, features2,
                            data1.num_pts, data2.num_pts, its.nfeatures, 0, nullptr, nullptr));
        CHECK(surfhip_device_synchronize());
        if (data1.h_data != NULL && data1.d_data != NULL && data1.num_pts > 0)
        {
            CHECK(surfhip_memcpy2d(&data1.h_data[0].score, sizeof(SurfPoint), &data1.d_data[0].score,
                                   sizeof(SurfPoint), 5 * sizeof(float), (size_t)data1.num_pts, SURFHIP_D2H));
        }
    }
}
