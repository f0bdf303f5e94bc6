/*
 * surfhip.h -- the C-ABI boundary of the MI355X SURF engine (libsurfhip.so).
 *
 * Plain C: plain pointers, sizes and int status codes; no HIP, torch or C++
 * types.  Device pointers are `void*`/typed pointers into HBM allocated with
 * surfhip_malloc (or by any HIP user in the same process, e.g. PyTorch).
 *
 * Every entry point names the reference interface it replaces (file:line in
 * the CUDA-SURF reference).  The C++ drop-in layer (include/surf.h,
 * include/cuda_utils.h, cuda-surf_amd/csrc/surf.cpp) is built only on these.
 */
#ifndef SURFHIP_H
#define SURFHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (replaces cudaError_t in CHECK(), cuda_utils.h:18-25) */
#define SURFHIP_OK               0
#define SURFHIP_ERR_INVALID     -1   /* bad argument / shape              */
#define SURFHIP_ERR_HIP         -2   /* HIP runtime error (see last error) */
#define SURFHIP_ERR_CAPACITY    -3   /* candidate buffer overflowed        */
#define SURFHIP_ERR_UNSUPPORTED -4   /* option outside the built path      */
#define SURFHIP_ERR_NOMEM       -5

/* copy kinds (cudaMemcpyKind) */
#define SURFHIP_H2H 0
#define SURFHIP_H2D 1
#define SURFHIP_D2H 2
#define SURFHIP_D2D 3

#ifdef __cplusplus
#define SURFHIP_BOOL bool
#else
#define SURFHIP_BOOL _Bool
#endif

/* Byte-identical to surf::SurfParam (surf_structures.h:45-72, 48 B). */
typedef struct surfhip_param {
    float thresh;
    int   init_lobe;
    SURFHIP_BOOL doubled;
    int   max_scale;
    int   noctaves;
    int   sampling;
    float divisor;
    SURFHIP_BOOL upright;
    SURFHIP_BOOL extend;
    int   desc_wsz;
    int   mag_factor;
    int   orient_size;
    int   nfeatures;
} surfhip_param;

/* Byte-identical to surf::SurfPoint (surf_structures.h:10-30, 48 B). */
typedef struct surfhip_point {
    float x, y, scale;
    int   o;
    float strength;
    int   laplace;
    float ori, score;
    int   match;
    float match_x, match_y, ambiguity;
} surfhip_point;

/* ------------------------------------------------------------ runtime --
 * Replaces cuda_utils.h:41-108 (initDevice, GpuTimer) and the cudart calls
 * main.cpp makes through it (main.cpp:16, 97, 100, 155, 219-226, 273-281). */
const char* surfhip_error_string(int status);     /* cudaGetErrorString      */
int  surfhip_last_hip_error(void);                /* raw hipError_t of the last failure */
int  surfhip_get_device_count(int* count);        /* cudaGetDeviceCount      */
int  surfhip_set_device(int dev);                 /* cudaSetDevice           */
int  surfhip_get_device(int* dev);
int  surfhip_device_name(int dev, char* buf, int len, int* cu_count);
int  surfhip_versions(int* driver, int* runtime); /* cudaDriver/RuntimeGetVersion */
int  surfhip_malloc(void** ptr, size_t bytes);    /* cudaMalloc              */
int  surfhip_malloc_pitch(void** ptr, size_t* pitch, size_t width_bytes, size_t height); /* cudaMallocPitch */
int  surfhip_free(void* ptr);                     /* cudaFree                */
int  surfhip_memset(void* ptr, int value, size_t bytes);             /* cudaMemset */
int  surfhip_memset_async(void* ptr, int value, size_t bytes, void* stream);
int  surfhip_memcpy(void* dst, const void* src, size_t bytes, int kind);  /* cudaMemcpy */
int  surfhip_memcpy_async(void* dst, const void* src, size_t bytes, int kind, void* stream);
int  surfhip_memcpy2d(void* dst, size_t dpitch, const void* src, size_t spitch,
                      size_t width_bytes, size_t height, int kind);     /* cudaMemcpy2D */
int  surfhip_device_synchronize(void);            /* cudaDeviceSynchronize   */
int  surfhip_device_reset(void);                  /* cudaDeviceReset         */
int  surfhip_stream_create(void** stream);
int  surfhip_stream_destroy(void* stream);
int  surfhip_stream_synchronize(void* stream);
int  surfhip_event_create(void** ev);             /* cudaEventCreate (GpuTimer) */
int  surfhip_event_destroy(void* ev);
int  surfhip_event_record(void* ev, void* stream);
int  surfhip_event_synchronize(void* ev);
int  surfhip_stream_wait_event(void* stream, void* ev);  /* cudaStreamWaitEvent */
int  surfhip_event_elapsed(float* ms, void* start, void* stop);

/* ----------------------------------------------------------- detector --
 * One detector = one geometry (W x H) + SurfParam + scratch for up to
 * max_batch frames, bound to one HIP stream.  Replaces the process-global
 * __constant__/__device__ state of surfd.cu:13-24 and the scratch members of
 * Surfor (surf.h:43-53), so several detectors (one per GPU / host thread)
 * can coexist. */
typedef struct surfhip_detector surfhip_detector;

/* Surfor::init + allocMemory (surf.cpp:60-91, 374-415).  `param` must come
 * from surfhip_make_param.  Frames up to 8,191 columns (after doubling) and
 * octave-0 sample grids below 16,384 x 16,384 (NMS record fields);
 * SURFHIP_ERR_UNSUPPORTED otherwise.  cand_cap = per-frame candidate capacity before
 * the canonical sort, rounded up to a power of 2 (0 = max(max_pts, 16384)).
 * stream = hipStream_t or NULL. */
int surfhip_detector_create(surfhip_detector** det, const surfhip_param* param,
                            int width, int height, int max_batch, int max_pts,
                            int cand_cap, void* stream);
int surfhip_detector_destroy(surfhip_detector* det);
int surfhip_detector_set_stream(surfhip_detector* det, void* stream);

/* Surfor::init parameter derivation (surf.cpp:63-79); returns
 * SURFHIP_ERR_UNSUPPORTED for max_scale != 5 or more than 128 features;
 * doubled = true doubles the sampling step and halves the divisor. */
int surfhip_make_param(surfhip_param* out, int noctaves, float thresh, int doubled,
                       int init_mask_size, int sampling_step, int upright,
                       int extend, int desc_wsz);

/* Batched detect+describe, asynchronous on the detector's stream.
 * Replaces the per-frame sequence cuIntegral (surfd.cu:2683) ->
 * cuHalfImage/cuCalcHessianMulti/cuFindMaximumWithInterp per octave
 * (surf.cpp:248-294, surfd.cu:2775, 2829, 3058) -> cuDescribe (surfd.cu:3251).
 *   d_frames : nframes u8 frames, row pitch `pitch` bytes (>= W, multiple of
 *              16), frame f at d_frames + f*frame_stride (16-B aligned)
 *   d_points : [nframes][max_pts] SurfPoint slots (device)
 *   d_desc   : [nframes][max_pts][nfeatures] f32 (device) or NULL (desc=false)
 *   d_counts : [nframes] int (device): keypoints kept per frame
 * Keypoints of a frame are in canonical order (octave, nms level, row, col);
 * descriptors are L2-normalised (surfd.cu:2447-2493). */
int surfhip_detect_batch(surfhip_detector* det, const uint8_t* d_frames, int nframes,
                         int pitch, size_t frame_stride, surfhip_point* d_points,
                         float* d_desc, int* d_counts);

/* detect_batch with the next batch's integral image computed on the
 * detector's side stream beside this batch's describe stage (software
 * pipelining across batches).  The next call that passes the same
 * next_frames (pointer, count, pitch, stride) as its `d_frames` uses the
 * prefetched integral instead of computing it.  next_frames must hold their
 * data when this call is made (in the detector stream's order) and stay
 * unchanged until that next call, or until surfhip_detector_drain; NULL =
 * detect_batch.  Doubled detectors compute every integral in line. */
int surfhip_detect_batch_next(surfhip_detector* det, const uint8_t* d_frames, int nframes,
                              int pitch, size_t frame_stride, surfhip_point* d_points,
                              float* d_desc, int* d_counts, const uint8_t* d_next_frames,
                              int next_nframes, int next_pitch, size_t next_frame_stride);

/* Orders the detector's side-stream work (a pending prefetch of the next
 * batch's integral, which reads next_frames) before anything later on the
 * detector's stream: after drain, synchronising that stream means
 * next_frames are no longer read.  The prefetch stays valid. */
int surfhip_detector_drain(surfhip_detector* det);

/* Record `event` (a surfhip_event_create / hipEvent_t) on the detector's
 * stream right before the describe stage of every following detect_batch /
 * detect_batch_next call (NULL: no longer).  A multi-GPU caller makes its
 * comm stream wait on it so the previous batch's all-gather lands beside the
 * latency-bound describe instead of the HBM-bound Hessian and NMS (SURVEY
 * 8e; no reference counterpart). */
int surfhip_detector_set_describe_event(surfhip_detector* det, void* event);

/* Surfor::detectAndCompute (surf.cpp:205-355) for one frame, synchronous.
 * Writes min(found, max_pts) SurfPoints to d_points, returns the count in
 * *num_pts; when desc != 0 allocates *d_desc_out = num_pts*nfeatures floats
 * (caller frees with surfhip_free, as main.cpp:275-282 does with cudaFree).
 * A frame with more NMS survivors than the candidate capacity returns
 * SURFHIP_OK with the first cand_cap survivors in scan order (as the
 * reference returns some max_pts points without a signal, surfd.cu:822-831):
 * callers that must know query surfhip_detector_status (the C++ Surfor
 * prints a warning). */
int surfhip_detect(surfhip_detector* det, const uint8_t* d_image, int pitch,
                   surfhip_point* d_points, int max_pts, int* num_pts,
                   float** d_desc_out, int desc);

/* Raw candidate count per frame of the last call (before the max_pts clamp,
 * surf.cpp:302-303); host array of nframes ints.  Returns
 * SURFHIP_ERR_CAPACITY (counts still written) when the last batch truncated
 * a frame at the candidate capacity. */
int surfhip_detector_candidates(surfhip_detector* det, int* h_counts, int nframes);

/* Did the last detect_batch / detect drop accepted candidates because a
 * frame had more NMS survivors than the candidate capacity (cand_cap of
 * surfhip_detector_create, rounded up to a power of 2)?  Such a frame keeps
 * its first cand_cap survivors in scan order -- deterministic -- sorted
 * canonically, then the first max_pts (the reference keeps an arbitrary
 * subset, surfd.cu:822-831).  The flag is reset by every batch. */
int surfhip_detector_status(surfhip_detector* det, int* truncated);
int surfhip_detector_capacity(surfhip_detector* det, int* cand_cap);

/* Stage timing (HIP events on the detector's stream) for the last
 * detect_batch: ms[0..5] = integral, hessian, nms, sort, describe, total. */
#define SURFHIP_NSTAGE 6
int surfhip_detector_set_profiling(surfhip_detector* det, int on);
int surfhip_detector_stage_times(surfhip_detector* det, float* ms);

/* In-step Hessian timing: with `on`, every following detect_batch records a
 * HIP event pair on the detector's stream around its Hessian launches, in
 * their normal (pipelined) arrangement -- the integral runs beside them on
 * the side stream -- for up to SURFHIP_MAX_HESS_EV batches.
 * surfhip_detector_hessian_times waits for them, writes the per-batch
 * milliseconds to ms[0..*n) and starts a new record. */
#define SURFHIP_MAX_HESS_EV 64
int surfhip_detector_time_hessian(surfhip_detector* det, int on);
int surfhip_detector_hessian_times(surfhip_detector* det, float* ms, int max, int* n);

/* Workspace access for parity tests: device pointers to frame 0's integral
 * image ((H+1) x ipitch int32, frame stride ii_stride ints) and response
 * planes (resp_stride floats per frame; octave o plane s at
 * ooff[o] + s*osize[o], row pitch swhp[o].z). */
int surfhip_detector_workspace(surfhip_detector* det, int32_t** d_ii, size_t* ii_stride,
                               float** d_resp, size_t* resp_stride);
int surfhip_detector_geometry(surfhip_detector* det, int* iwhp /*3*/, int* swhp /*3*8*/,
                              long long* ooff /*8*/, int* osize /*8*/);

/* Stage-level entry points on frames already resident (parity tests and the
 * Hessian roofline run): integral only, Hessian only.  run_hessian needs a
 * prior run_integral (or detect_batch) on frames that are still live: the
 * u8 Hessian kernels re-read those frames (SURFHIP_ERR_INVALID if there were
 * none). */
int surfhip_run_integral(surfhip_detector* det, const uint8_t* d_frames, int nframes,
                         int pitch, size_t frame_stride);
int surfhip_run_hessian(surfhip_detector* det, int nframes);

/* Algorithmic (compulsory) HBM bytes per frame of the Hessian stage:
 * integral image read once + valid responses written. */
long long surfhip_hessian_bytes_per_frame(surfhip_detector* det);

/* The Hessian stage's kernels for this detector's launch plan, as text
 * (e.g. "k_hess_q0 (octave 0) + k_hess_v1 (octave 1) + k_hess_far (octaves
 * 2-3)"), NUL-terminated in buf[len]; returns the full length. */
int surfhip_hessian_plan(surfhip_detector* det, char* buf, int len);

/* Result slab for the multi-GPU all-gather, compacted to the
 * keypoints actually found by the last detect_batch:
 *   int32 {nframes, total, nfeatures (0 without descriptors), flags}
 *     (flags bit 0: a frame was truncated at the candidate capacity;
 *      bit 1: the slab exceeded surfhip_pack_slab_cap's capacity)
 *   int32 counts[nframes] padded to 16 B
 *   SurfPoint points[total]          (frame-major, canonical order)
 *   float desc[total][nfeatures]
 * surfhip_batch_total synchronises the stream and returns the batch's total
 * keypoint count (needed to size the collective). */
size_t surfhip_slab_bytes(int nframes, int total, int nfeatures);
int surfhip_batch_total(surfhip_detector* det, int nframes, int* total);
int surfhip_pack_slab(surfhip_detector* det, const surfhip_point* d_points, const float* d_desc,
                      const int* d_counts, int nframes, void* d_slab);
/* Both pack functions read the detector's per-batch offsets and status
 * word: enqueue them on the detector's stream BEFORE the next detect_batch
 * (which resets both), as bench.py and the ingest ring do.
 * The same into a buffer of cap_bytes, with no host synchronisation: the
 * multi-GPU path sizes every rank's slab once (a per-frame keypoint budget,
 * SURVEY.md 8e) and all-gathers that many bytes per batch.  A batch that
 * does not fit writes its header and counts with flags bit 1 set and no
 * payload; the receiver must check the flags. */
int surfhip_pack_slab_cap(surfhip_detector* det, const surfhip_point* d_points, const float* d_desc,
                          const int* d_counts, int nframes, void* d_slab, size_t cap_bytes);

/* ------------------------------------------------------------ matching --
 * Surfor::match (surf.cpp:418-428) -> cuFindMaxCorr (surfd.cu:3554-3566) ->
 * findMaxCorr (surfd.cu:2530-2656), asynchronous on `stream` (NULL = the
 * null stream).  For each of the n1 points of set 1 writes score (best dot
 * product), match (index into set 2, -1 when no score is positive),
 * match_x/match_y (that point's x, y; 0 for -1) and ambiguity
 * (second / (best + 1e-6)) -- the reference's per-thread-row top-2 and row
 * merge, bit-exact.  Descriptors: n x nfeatures f32 rows (nfeatures a
 * multiple of 4, <= 128).  flags: SURFHIP_MATCH_FULL_TAIL also scores the
 * last partial 32-point tile of set 2, which the reference drops
 * (surfd.cu:2569); 0 follows the reference.  Scratch (surfhip_match_scratch
 * bytes, device) is caller-provided (the call is then asynchronous), or
 * NULL: the library allocates it and the call returns after the stream has
 * finished the match. */
#define SURFHIP_MATCH_FULL_TAIL 1
size_t surfhip_match_scratch(int n1, int n2, int flags);
int surfhip_match(surfhip_point* d_pts1, const surfhip_point* d_pts2, const float* d_feat1,
                  const float* d_feat2, int n1, int n2, int nfeatures, int flags,
                  void* d_scratch, void* stream);

/* ------------------------------------------------------------- ingest --
 * Pipelined host-frame ingest.  Replaces the
 * per-frame blocking cudaMemcpy2D of a pageable frame (main.cpp:212-226) and
 * the blocking per-frame point copy-back (surf.cpp:335-342) with a ring of
 * `depth` pinned host frame slots / HBM frame slots / result slabs:
 *   acquire  -> pinned u8 slot [max_batch][H][pitch], pitch = align128(W)
 *               (SURFHIP_ERR_CAPACITY when `depth` batches await collect)
 *   submit   -> H2D on a copy stream, detect+describe on the detector's
 *               stream after that copy only, pack into the slot's slab
 *   collect  -> oldest batch's compacted result slab (format above) in
 *               pinned host memory, valid until that slot is collected again
 * Results are bit-identical to surfhip_detect_batch + surfhip_pack_slab. */
#define SURFHIP_INGEST_MAX_DEPTH 8
typedef struct surfhip_ingest surfhip_ingest;
int surfhip_ingest_create(surfhip_ingest** ing, surfhip_detector* det, int depth);
int surfhip_ingest_destroy(surfhip_ingest* ing);
int surfhip_ingest_acquire(surfhip_ingest* ing, uint8_t** h_frames, int* pitch, size_t* frame_stride);
int surfhip_ingest_submit(surfhip_ingest* ing, int nframes);
int surfhip_ingest_collect(surfhip_ingest* ing, const void** h_slab, size_t* bytes);
int surfhip_ingest_pending(surfhip_ingest* ing, int* n);

/* --------------------------------------------------------------- dump --
 * On-disk keypoint + descriptor file (no reference counterpart: main.cpp
 * only draws the points, main.cpp:21-71).  A file is a sequence of records;
 * a record is this 64-B little-endian header followed by slab_bytes of one
 * result slab exactly as surfhip_pack_slab / surfhip_ingest_collect return
 * it.  surfhip_dump_append appends one record (creating the file). */
#define SURFHIP_DUMP_MAGIC "SURFKPD1"
#define SURFHIP_DUMP_VERSION 1
typedef struct surfhip_dump_header {
    char     magic[8];              /* "SURFKPD1"                         */
    uint32_t header_bytes;          /* 64                                 */
    uint32_t version;               /* 1                                  */
    uint32_t width, height;         /* frame size                         */
    uint32_t nframes, nfeatures;    /* nfeatures 0: no descriptors        */
    uint64_t total;                 /* keypoints in the slab              */
    uint64_t slab_bytes;            /* bytes following this header       */
    uint64_t first_frame;           /* caller's index of the first frame  */
    float    thresh;
    uint8_t  noctaves, upright, extend, doubled;
} surfhip_dump_header;
int surfhip_dump_append(const char* path, const void* h_slab, size_t bytes, int width, int height,
                        const surfhip_param* param, long long first_frame);

/* Measured HBM stream rates (SURVEY 8d "also report measured peak from an
 * in-repo stream-copy kernel"; no reference counterpart).  One launch of a
 * 16-B-per-lane streaming kernel over `bytes` (a multiple of 16, src and dst
 * 16-B aligned) on `stream`, all 256 CUs, grid-stride:
 *   mode 0 copy  src -> dst  (moves 2 x bytes: read + write)
 *   mode 1 read  src only    (dst written only if a running XOR hits a
 *                             64-bit magic: never, for practical data)
 *   mode 2 write dst only    (writes bytes)
 * The caller times launches with events; surfhip_stream_bytes gives the HBM
 * bytes one launch of a mode moves. */
int surfhip_stream_run(int mode, const void* src, void* dst, size_t bytes, void* stream);
size_t surfhip_stream_bytes(int mode, size_t bytes);

/* Library build identification (for the loaded-.so audit). */
const char* surfhip_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* SURFHIP_H */
