// surf_structures.h -- public SURF data types, layout-compatible with the
// CUDA-SURF reference (surf_structures.h:7-72 there).
//
// Offsets are part of the drop-in contract (the D2H copy in
// Surfor::detectAndCompute moves the first 6/7 4-byte fields of each point,
// surf.cpp:335-342 in the reference) and are static_assert-ed below.
#pragma once

#include <cstddef>

namespace surf
{
    // One interest point (48 bytes).
    struct SurfPoint
    {
        float x = -1;          // 0   image column
        float y = -1;          // 4   image row
        float scale = 1;       // 8   detected scale
        int o = 0;             // 12  octave index (written by this engine)
        float strength = 0;    // 16  interpolated Hessian response
        int laplace = 1;       // 20  sign of the Laplacian (+1 / -1)
        float ori = 0;         // 24  orientation (radians; 0 when upright)
        float score = 0;       // 28  match score            (Surfor::match)
        int match = -1;        // 32  index of matched point (Surfor::match)
        float match_x = 0;     // 36
        float match_y = 0;     // 40
        float ambiguity = 0;   // 44  second best / best score
    };

    // A set of points on host and device (24 bytes).
    struct SurfData
    {
        int num_pts;           // points currently held
        int max_pts;           // capacity of h_data / d_data
        SurfPoint* h_data;     // host copy (fields x..laplace[, ori])
        SurfPoint* d_data;     // device array (HBM)
    };

    // Detector parameters as Surfor::init derives them (48 bytes).
    struct SurfParam
    {
        float thresh;          // 0   blob response threshold
        int init_lobe;         // 4   initial lobe size (init_mask_size / 3)
        bool doubled;          // 8   double the image first (not supported here)
        int max_scale;         // 12  scales per octave (init_lobe + 2)
        int noctaves;          // 16
        int sampling;          // 20  initial sampling step
        float divisor;         // 24  coordinate factor (0.5 when doubled)
        bool upright;          // 28  U-SURF when true
        bool extend;           // 29  128-D descriptor when true
        int desc_wsz;          // 32  descriptor window cells per side
        int mag_factor;        // 36  12 / desc_wsz
        int orient_size;       // 40  4 or 8 bins per cell
        int nfeatures;         // 44  desc_wsz^2 * orient_size
    };

    static_assert(sizeof(SurfPoint) == 48, "SurfPoint must be 48 bytes");
    static_assert(offsetof(SurfPoint, o) == 12 && offsetof(SurfPoint, laplace) == 20 &&
                  offsetof(SurfPoint, ori) == 24 && offsetof(SurfPoint, ambiguity) == 44,
                  "SurfPoint field offsets");
    static_assert(sizeof(SurfData) == 24 && offsetof(SurfData, d_data) == 16, "SurfData layout");
    static_assert(sizeof(SurfParam) == 48 && offsetof(SurfParam, doubled) == 8 &&
                  offsetof(SurfParam, upright) == 28 && offsetof(SurfParam, extend) == 29 &&
                  offsetof(SurfParam, nfeatures) == 44,
                  "SurfParam layout");
}
