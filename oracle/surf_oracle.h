/*
 * surf_oracle.h -- CPU restatement of the CUDA-SURF detect+describe path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libsurfhip, libsurf,
 * bench.py's GPU leg) may link, call or execute this code.  It is the checker
 * the parity tests compare the HIP path against, and the CPU baseline that
 * bench.py times beside the GPU.
 *
 * PARITY STATUS: "parity unpinned" against the reference binary.  The
 * reference (surfd.cu) needs nvcc + an NVIDIA GPU and cannot be built or run
 * here, and the reference ships no golden outputs, known-answer tests or
 * fixtures.  This oracle restates the reference source
 * line by line (citations per function) with floating-point contraction OFF
 * and explicit fmaf() exactly where the reference wrote __fmaf_rn.  It is
 * pinned by (a) closed-form known-answer tests (tests/test_oracle.py) and
 * (b) the only reference data files, data/left.pgm and data/right.pgm, whose
 * outputs are frozen as golden vectors under tests/golden/.
 *
 * Deliberate, documented deviations from the reference (all are reference
 * bugs or nondeterminism, see DESIGN.md section "Fixed semantics"):
 *   - row 0 / column 0 of the integral image are written as zeros (the
 *     reference relies on a memset of the previous call, surf.cpp:347);
 *   - SurfPoint.o is written with the octave index (never written in the
 *     reference, surfd.cu:1001-1022);
 *   - the per-octave point counter never restarts (surfd.cu:825-826 restarts
 *     at 0 when an octave emits nothing);
 *   - emission order is canonical (octave, nms level, block row, block col)
 *     and the max_pts cap keeps the first max_pts in that order (the
 *     reference emits in atomicInc order and has no pi<max guard,
 *     surfd.cu:827-830);
 *   - float histogram/descriptor sums are accumulated in sample order (the
 *     reference uses unordered float atomics, surfd.cu:1222-1266, 1795-1905);
 *   - __sinf/__cosf (surfd.cu:2423-2424) are replaced by surf_sinf/surf_cosf,
 *     a fixed polynomial of plain float ops that the HIP kernels evaluate
 *     identically.
 */
#ifndef SURF_ORACLE_H
#define SURF_ORACLE_H

#include <stdint.h>
#include <stddef.h>
#include <stdbool.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Byte-identical to surf::SurfPoint (surf_structures.h:10-30): 48 bytes. */
typedef struct {
    float x, y, scale;
    int   o;
    float strength;
    int   laplace;
    float ori, score;
    int   match;
    float match_x, match_y, ambiguity;
} or_point;

/* Byte-identical to surf::SurfParam (surf_structures.h:45-72): 48 bytes. */
typedef struct {
    float thresh;
    int   init_lobe;
    bool  doubled;
    int   max_scale;
    int   noctaves;
    int   sampling;
    float divisor;
    bool  upright;
    bool  extend;
    int   desc_wsz;
    int   mag_factor;
    int   orient_size;
    int   nfeatures;
} or_param;

#define OR_MAX_OCTAVE 8
#define OR_MAX_SCALE  8
#define OR_NBIN       72

typedef struct { int x, y, z; } or_int3;

/* Geometry of one frame (surf.cpp:374-392). */
typedef struct {
    or_int3 iwhp;                     /* integral: (W+1, H+1, align128(W+1)) */
    or_int3 swhp[OR_MAX_OCTAVE];      /* response grid per octave            */
    int     osize[OR_MAX_OCTAVE];     /* sh * sp floats per plane            */
    size_t  ooff[OR_MAX_OCTAVE];      /* float offset of octave o's plane 0  */
    size_t  tot_osize;                /* floats, all octaves x max_scale     */
} or_geom;

/* Per-octave Hessian / NMS parameters exactly as the reference host code
 * derives them (surf.cpp:240-292, surfd.cu:2829-2865, 3058-3071). */
typedef struct {
    int octave;                       /* 1, 2, 4, ...                        */
    int init_scale;                   /* 0 for o == 0, 2 otherwise           */
    int nscale;                       /* max_scale - init_scale              */
    int delta;                        /* sampling * octave                   */
    int mask[OR_MAX_SCALE];           /* indexed by i = s - init_scale       */
    int border1[OR_MAX_SCALE];        /* Hessian valid border, index i       */
    int x2[OR_MAX_SCALE], x3[OR_MAX_SCALE], x4[OR_MAX_SCALE];
    float norm[OR_MAX_SCALE];
    int borders[OR_MAX_SCALE];        /* host borders[] (d_borders), index s */
    int mborders[3];                  /* NMS start offsets (maximum_borders[(MAX_SCALE - 2) / 2]) */
    int nms_gx, nms_gy;               /* NMS launch extent in threads        */
} or_octave;

/* Surfor::init (surf.cpp:60-91).  Returns 0, or -1 for unsupported options
 * (max_scale != 5: the NMS levels assume 5 scales per octave). */
int  or_init_param(or_param* p, int noctaves, float thresh, bool doubled,
                   int init_mask_size, int sampling_step, bool upright,
                   bool extend, int desc_wsz);
/* Surfor::initLut (surf.cpp:358-371) and the orientation bins (surf.cpp:83-89). */
void or_init_tables(float lut1[83], float lut2[40], float bins[OR_NBIN]);
/* Surfor::allocMemory sizes (surf.cpp:374-392). */
void or_geometry(const or_param* p, int w, int h, or_geom* g);
/* Host parameter recurrences for every octave. */
void or_octave_params(const or_param* p, const or_geom* g, or_octave oct[OR_MAX_OCTAVE]);

/* integralRow + integralCol (surfd.cu:129-165): ii is (H+1) x ipitch int32. */
void or_integral(const uint8_t* img, int w, int h, int pitch,
                 int32_t* ii, int ipitch);
/* The doubled image D of cuIntegralDoubleU4 (surfd.cu:166-318, 2707-2772):
 * (2w-2) x (2h-2) u8, row pitch dpitch; integral(D) is the reference's
 * doubled integral image. */
void or_double_image(const uint8_t* img, int w, int h, int pitch, uint8_t* dst, int dpitch);
/* All response planes of all octaves (halfImage + calcHessianMultiConst,
 * surf.cpp:248-294, surfd.cu:321-331, 445-481).  resp has g->tot_osize floats
 * and is fully overwritten (zeros outside each scale's valid window). */
void or_hessian(const or_param* p, const or_geom* g, const or_octave* oct,
                const int32_t* ii, float* resp);

/* Non-max suppression + interpolation + makePoint for all octaves
 * (findMaximumWithInterp, surfd.cu:676-832, 942-1022).  Writes at most
 * max_pts points in canonical order; returns the number of candidates found
 * (may exceed max_pts; the caller clamps like surf.cpp:303). */
int  or_find_points(const or_param* p, const or_geom* g, const or_octave* oct,
                    const int32_t* ii, const float* resp,
                    or_point* pts, int max_pts);

/* Orientation (assignOrientationApprox, surfd.cu:1711-1960). */
float or_orientation(const or_param* p, const or_geom* g, const int32_t* ii,
                     const float lut1[83], const float bins[OR_NBIN],
                     const or_point* pt);
/* Descriptor without normalization (surfd.cu:1566-1615 upright,
 * 2391-2444 rotated) followed by normalize (surfd.cu:2447-2493). */
void or_describe(const or_param* p, const or_geom* g, const int32_t* ii,
                 const float lut2[40], const or_point* pt, float* desc);

/* Whole detectAndCompute on one frame (surf.cpp:205-355).  desc may be NULL
 * (desc=false).  Returns num_pts (<= max_pts). */
int  or_detect_and_compute(const or_param* p, const uint8_t* img, int w, int h,
                           int pitch, or_point* pts, int max_pts, float* desc,
                           int* n_candidates);

/* Surfor::match / findMaxCorr (surf.cpp:418-428, surfd.cu:2530-2656):
 * writes score, match, match_x, match_y, ambiguity of pts1[0..n1). */
void or_match(or_point* pts1, const or_point* pts2, const float* f1, const float* f2,
              int n1, int n2, int nf, int full_tail);

/* Deterministic sine/cosine used in place of __sinf/__cosf. */
/* test infrastructure: mismatches of the kernels' x * r + remainder quotient */
long or_div_by_mismatches(long n, uint64_t seed);
float or_sinf(float x);
float or_cosf(float x);
/* dFastAtan2 (surfd.cu:114-126). */
float or_fast_atan2(float y, float x);

/* CPU baseline: run or_detect_and_compute over nframes frames with nthreads
 * threads; returns wall seconds (frame generation excluded). */
double or_bench_frames(const or_param* p, const uint8_t* frames, int nframes,
                       int w, int h, int pitch, size_t frame_stride,
                       int max_pts, int nthreads, long long* total_pts);

/* Known-answer-test hooks on internal steps. */
void     or_test_solve3(float sol[3], float sq[9]);   /* solveLinearSystem */
float    or_test_fit(const float* src, float off[3], int s, int r, int c, int osize, int sp); /* fitQuadrat */
uint32_t or_test_box(const int32_t* ii, int ipitch, int x1, int y1, int x2, int y2); /* getSum */
void     or_test_place(float* desc, int wsz, int osz, float mag1, int ori1, float mag2, int ori2,
                       float rx, float cx);             /* placeInIndex */

#ifdef __cplusplus
}
#endif
#endif
