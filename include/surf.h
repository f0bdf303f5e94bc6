// surf.h -- public C++ API of the SURF engine, source-compatible with the
// CUDA-SURF reference's surf.h:7-63 (same namespace, class, member functions,
// argument meanings and defaults).  Implemented in cuda-surf_amd/csrc/surf.cpp
// (libsurf.so) on top of the libsurfhip C-ABI.
#pragma once
#include "surf_structures.h"
#include "cuda_utils.h"

struct surfhip_detector;

namespace surf
{
    /* Allocate max_pts points on host (malloc) and/or device (HBM). */
    void initSurfData(SurfData& data, const int max_pts, const bool host, const bool dev);

    /* Free what initSurfData allocated. */
    void freeSurfData(SurfData& data);

    /***** SURF detector *****/
    class Surfor
    {
    public:
        Surfor();
        ~Surfor();

        /* Parameters (surf.h:27-29 of the reference); doubled=true upsamples the
         * frame 2x before the integral (surf.cpp:234, 377-378) and describes at
         * (2x, 2y), 3.3*scale (surfd.cu:1581-1592). */
        void init(const int _noctaves, const float _thresh = 0.2f, const bool _doubled = false,
                  const int _init_mask_size = 9, const int _sampling_step = 2, const bool _upright = false,
                  const bool _extend = false, const int _desc_wsz = 4, const int _width = -1,
                  const int _height = -1);

        /* Detect keypoints of a device u8 image (row pitch whp0.z bytes) into
         * result, and -- when desc -- allocate *desc_addr = num_pts x nfeatures
         * device floats (caller frees with cudaFree). */
        void detectAndCompute(unsigned char* image, SurfData& result, int3 whp0, float** desc_addr,
                              const bool desc = true);

        /* Descriptor matching (reference surf.cpp:418-428): for each point of
         * data1 the best (score, match, match_x, match_y, ambiguity) over
         * data2 on the device (surfhip_match), copied to data1.h_data. */
        void match(SurfData& data1, SurfData& data2, float* features1, float* features2);

    private:
        SurfParam its{};
        int3 whp{0, 0, 0};
        surfhip_detector* det = nullptr;      // scratch sized for (whp.x, whp.y)
        int det_w = 0, det_h = 0, det_pts = 0;
        bool warned_trunc = false;            // candidate-capacity truncation reported
    };
}
