// surfhip_api.hip -- the C-ABI of libsurfhip.so (declared in include/surfhip.h).
//
// Host orchestration of the detect+describe path.  The reference does this
// per frame in Surfor::detectAndCompute (surf.cpp:205-355) with 22 symbol
// uploads, 4 blocking syncs, a cudaMalloc and two scratch memsets per frame;
// here a detector derives every parameter once at creation, owns HBM scratch
// for a whole batch of frames, and enqueues ~14 launches per batch on its own
// stream with no host synchronisation.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "surfhip.h"
#include "surfhip_internal.h"

using namespace surfhip;

static_assert(sizeof(surfhip_point) == 48, "SurfPoint layout (surf_structures.h:10-30)");
static_assert(sizeof(surfhip_param) == 48, "SurfParam layout (surf_structures.h:45-72)");
static_assert(offsetof(surfhip_param, doubled) == 8 && offsetof(surfhip_param, upright) == 28 &&
              offsetof(surfhip_param, extend) == 29 && offsetof(surfhip_param, nfeatures) == 44,
              "SurfParam field offsets");
static_assert(offsetof(surfhip_point, o) == 12 && offsetof(surfhip_point, laplace) == 20 &&
              offsetof(surfhip_point, ori) == 24 && offsetof(surfhip_point, ambiguity) == 44,
              "SurfPoint field offsets");

static_assert(sizeof(surfhip_dump_header) == 64, "dump record header");

static thread_local hipError_t g_last_hip = hipSuccess;

#define HIPCHK(x)                                    \
    do {                                             \
        hipError_t e_ = (x);                         \
        if (e_ != hipSuccess) {                      \
            g_last_hip = e_;                         \
            return SURFHIP_ERR_HIP;                  \
        }                                            \
    } while (0)

static inline int align_up(int a, int b) { return (a % b != 0) ? (a - a % b + b) : a; }  // cuda_utils.h:160-163

struct surfhip_detector {
    int dev = 0;
    int cus = 256;                      // compute units of dev (the describe kernels' persistent grid)
    hipStream_t stream = nullptr;
    surfhip_param param{};
    FrameParams P{};
    OctaveParams oct[kMaxOct]{};
    OctaveParams* d_oct = nullptr;      // device copy read by the fused launches
    LaunchPlan plan{};
    int W = 0, H = 0, max_batch = 0, max_pts = 0, cap = 0;   // W x H: the frames the integral is taken of
    int srcW = 0, srcH = 0;             // the caller's frames (= W x H unless doubled)
    uint8_t* dbl = nullptr;             // doubled: the (2 srcW - 2) x (2 srcH - 2) frames D
    int dpitch = 0;
    long long dstride = 0;
    int nbands = 0, CW = 0;
    size_t tot_osize = 0;
    int32_t* ii = nullptr;              // integral of the last processed batch (one of iib)
    int32_t* iib[2] = {nullptr, nullptr};   // integral buffers: the batch's, and the next batch's prefetch
    int icur = 0;                       // iib index of ii
    // prefetched integral (surfhip_detect_batch_next): which frames, in iib[ipref]
    bool pref_valid = false;
    int ipref = 0, pref_n = 0, pref_pitch = 0;
    const uint8_t* pref_frames = nullptr;
    size_t pref_stride = 0;
    hipEvent_t fork2 = nullptr;
    float* resp = nullptr;
    uint32_t* colsum = nullptr;
    // plan.iiw: k_ii_rowseg's row sums of the batch (or of the next batch,
    // prefetched) that k_hess_w adds to its strip integrals
    uint32_t* rowseg = nullptr;
    surfhip_point* cand = nullptr;
    uint32_t* keys = nullptr;
    uint64_t* gscratch = nullptr;
    int* cand_count = nullptr;
    uint32_t* scan_key = nullptr;       // NMS survivors awaiting interpolation
    uint32_t* scan_src = nullptr;
    float* scan_cube = nullptr;         // the survivors' fit inputs (kCubeCap per scan item)
    int* item_count = nullptr;          // survivors per NMS scan item
    int* item_off = nullptr;            // their exclusive prefix (+ total)
    int nitems = 0;                     // scan items per frame
    int* offsets = nullptr;
    int* order = nullptr;               // per frame: keypoint indices in row order (describe schedule)
    float4* work = nullptr;             // the describe schedule flattened: kWorkF4 float4 per keypoint (k_worklist)
    int* status = nullptr;
    // single-frame API slots
    surfhip_point* pts1 = nullptr;
    float* desc1 = nullptr;
    int* count1 = nullptr;
    bool profiling = false;
    hipEvent_t ev[SURFHIP_NSTAGE]{};
    hipStream_t side = nullptr;         // integral + integral-image Hessian kernels, beside the u8 ones
    hipEvent_t fork = nullptr, join = nullptr;
    float stage_ms[SURFHIP_NSTAGE]{};
    bool time_hess = false;             // in-step Hessian event pairs (surfhip_detector_time_hessian)
    // per timed batch: [0] on the detector stream before the Hessian's fork,
    // [1] on it after the u8 kernels, [2] on the side stream after the
    // integral-image kernels (only when the plan has some: hev_side)
    hipEvent_t hev[SURFHIP_MAX_HESS_EV][3]{};
    hipEvent_t desc_ev = nullptr;       // caller's event, recorded before each describe stage
    bool hev_side[SURFHIP_MAX_HESS_EV]{};
    int hev_n = 0;
    int last_nframes = 0;
    const uint8_t* last_frames = nullptr;   // u8 source of the last integral (surfhip_run_hessian)
    int last_pitch = 0;
    long long last_fstride = 0;
    long long hess_bytes = 0;
};

extern "C" {

// ---------------------------------------------------------------- runtime

const char* surfhip_error_string(int status)
{
    switch (status) {
        case SURFHIP_OK: return "no error";
        case SURFHIP_ERR_INVALID: return "invalid argument";
        case SURFHIP_ERR_HIP: return hipGetErrorString(g_last_hip);
        case SURFHIP_ERR_CAPACITY: return "candidate capacity exceeded";
        case SURFHIP_ERR_UNSUPPORTED: return "unsupported option";
        case SURFHIP_ERR_NOMEM: return "out of memory";
        default: return "unknown error";
    }
}

int surfhip_last_hip_error(void) { return (int)g_last_hip; }

int surfhip_get_device_count(int* count)
{
    HIPCHK(hipGetDeviceCount(count));
    return SURFHIP_OK;
}
int surfhip_set_device(int dev)
{
    HIPCHK(hipSetDevice(dev));
    return SURFHIP_OK;
}
int surfhip_get_device(int* dev)
{
    HIPCHK(hipGetDevice(dev));
    return SURFHIP_OK;
}
int surfhip_device_name(int dev, char* buf, int len, int* cu_count)
{
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, dev));
    if (buf && len > 0) {
        snprintf(buf, (size_t)len, "%s (%s)", prop.name, prop.gcnArchName);
    }
    if (cu_count) *cu_count = prop.multiProcessorCount;
    return SURFHIP_OK;
}
int surfhip_versions(int* driver, int* runtime)
{
    HIPCHK(hipDriverGetVersion(driver));
    HIPCHK(hipRuntimeGetVersion(runtime));
    return SURFHIP_OK;
}
int surfhip_malloc(void** ptr, size_t bytes)
{
    HIPCHK(hipMalloc(ptr, bytes));
    return SURFHIP_OK;
}
int surfhip_malloc_pitch(void** ptr, size_t* pitch, size_t width_bytes, size_t height)
{
    HIPCHK(hipMallocPitch(ptr, pitch, width_bytes, height));
    return SURFHIP_OK;
}
int surfhip_free(void* ptr)
{
    HIPCHK(hipFree(ptr));
    return SURFHIP_OK;
}
int surfhip_memset(void* ptr, int value, size_t bytes)
{
    HIPCHK(hipMemset(ptr, value, bytes));
    return SURFHIP_OK;
}
int surfhip_memset_async(void* ptr, int value, size_t bytes, void* stream)
{
    HIPCHK(hipMemsetAsync(ptr, value, bytes, (hipStream_t)stream));
    return SURFHIP_OK;
}
static hipMemcpyKind kind_of(int k)
{
    switch (k) {
        case SURFHIP_H2H: return hipMemcpyHostToHost;
        case SURFHIP_H2D: return hipMemcpyHostToDevice;
        case SURFHIP_D2H: return hipMemcpyDeviceToHost;
        case SURFHIP_D2D: return hipMemcpyDeviceToDevice;
        default: return hipMemcpyDefault;
    }
}
int surfhip_memcpy(void* dst, const void* src, size_t bytes, int kind)
{
    HIPCHK(hipMemcpy(dst, src, bytes, kind_of(kind)));
    return SURFHIP_OK;
}
int surfhip_memcpy_async(void* dst, const void* src, size_t bytes, int kind, void* stream)
{
    HIPCHK(hipMemcpyAsync(dst, src, bytes, kind_of(kind), (hipStream_t)stream));
    return SURFHIP_OK;
}
int surfhip_memcpy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width_bytes,
                     size_t height, int kind)
{
    HIPCHK(hipMemcpy2D(dst, dpitch, src, spitch, width_bytes, height, kind_of(kind)));
    return SURFHIP_OK;
}
int surfhip_device_synchronize(void)
{
    HIPCHK(hipDeviceSynchronize());
    return SURFHIP_OK;
}
int surfhip_device_reset(void)
{
    HIPCHK(hipDeviceReset());
    return SURFHIP_OK;
}
int surfhip_stream_create(void** stream)
{
    hipStream_t s;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = (void*)s;
    return SURFHIP_OK;
}
int surfhip_stream_destroy(void* stream)
{
    HIPCHK(hipStreamDestroy((hipStream_t)stream));
    return SURFHIP_OK;
}
int surfhip_stream_synchronize(void* stream)
{
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    return SURFHIP_OK;
}
int surfhip_event_create(void** ev)
{
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    *ev = (void*)e;
    return SURFHIP_OK;
}
int surfhip_event_destroy(void* ev)
{
    HIPCHK(hipEventDestroy((hipEvent_t)ev));
    return SURFHIP_OK;
}
int surfhip_event_record(void* ev, void* stream)
{
    HIPCHK(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream));
    return SURFHIP_OK;
}
int surfhip_stream_wait_event(void* stream, void* ev)
{
    HIPCHK(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev, 0));
    return SURFHIP_OK;
}
int surfhip_event_synchronize(void* ev)
{
    HIPCHK(hipEventSynchronize((hipEvent_t)ev));
    return SURFHIP_OK;
}
int surfhip_event_elapsed(float* ms, void* start, void* stop)
{
    HIPCHK(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
    return SURFHIP_OK;
}

// --------------------------------------------------------------- detector

// Surfor::init (surf.cpp:63-79).
int surfhip_make_param(surfhip_param* out, int noctaves, float thresh, int doubled, int init_mask_size,
                       int sampling_step, int upright, int extend, int desc_wsz)
{
    if (!out) return SURFHIP_ERR_INVALID;
    memset(out, 0, sizeof(*out));
    if (noctaves < 1 || noctaves > kMaxOct || desc_wsz < 1 || sampling_step < 1)
        return SURFHIP_ERR_INVALID;
    out->doubled = doubled != 0;
    out->noctaves = noctaves;
    out->divisor = doubled ? 0.5f : 1.f;
    out->init_lobe = init_mask_size / 3;
    out->max_scale = out->init_lobe + 2;
    out->sampling = sampling_step + (doubled ? sampling_step : 0);
    out->thresh = thresh;
    out->upright = upright != 0;
    out->extend = extend != 0;
    out->desc_wsz = desc_wsz;
    out->mag_factor = 12 / desc_wsz;
    out->orient_size = 4 + (extend ? 4 : 0);
    out->nfeatures = desc_wsz * desc_wsz * out->orient_size;
    // scales per octave: MAX_SCALE (surfd.h:9) bounds them; below 4 the
    // octaves > 0 compute fewer than 2 scales and the lobes degenerate
    if (out->max_scale < 4 || out->max_scale > kMaxScale) return SURFHIP_ERR_UNSUPPORTED;
    // a sample's Gaussian weight is lookup2[(int)(rpos^2 + cpos^2)]
    // (surfd.cu:1303, 1335, 1999) with |rpos|, |cpos| < (desc_wsz + 1) / 2,
    // and lookup2 has 40 entries (surfd.cu:23): from desc_wsz 8 on the
    // reference reads past it.  desc_wsz <= 7: at most 7 x 7 x 8 = 392 features.
    if (desc_wsz > 7) return SURFHIP_ERR_UNSUPPORTED;
    return SURFHIP_OK;
}

// Geometry (surf.cpp:374-392) and the host parameter recurrences
// (surf.cpp:240-292, surfd.cu:2844-2865, 3062-3076).
static int derive(surfhip_detector* d)
{
    const surfhip_param& p = d->param;
    FrameParams& P = d->P;
    P.W = d->W;
    P.H = d->H;
    const int iw = d->W + 1, ih = d->H + 1;
    P.ip = align_up(iw, 128);
    P.iH = ih;
    P.ii_stride = (long long)ih * P.ip;
    P.max_scale = p.max_scale;
    P.init_lobe = p.init_lobe;
    P.sampling = p.sampling;
    P.noct = p.noctaves;
    P.thresh = p.thresh;
    P.divisor = p.divisor;
    P.upright = p.upright;
    P.extend = p.extend;
    P.wsz = p.desc_wsz;
    P.mag = p.mag_factor;
    P.osz = p.orient_size;
    P.nfeat = p.nfeatures;
    P.doubled = p.doubled ? 1 : 0;

    int sw[kMaxOct], sh[kMaxOct], sp[kMaxOct];
    long long off = 0;
    for (int o = 0; o < p.noctaves; o++) {
        sw[o] = o == 0 ? (iw - 1) / p.sampling : sw[o - 1] >> 1;
        sh[o] = o == 0 ? (ih - 1) / p.sampling : sh[o - 1] >> 1;
        sp[o] = align_up(std::max(sw[o], 1), 128);
        OctaveParams& q = d->oct[o];
        q.sw = sw[o];
        q.sh = sh[o];
        q.sp = sp[o];
        q.osize = sh[o] * sp[o];
        q.ooff = off;
        off += (long long)q.osize * p.max_scale;
    }
    P.resp_stride = off;
    d->tot_osize = (size_t)off;

    int mask_size = p.init_lobe - 2;
    int octave = 1;
    int borders[kMaxScale] = {0};
    long long hbytes = 0;
    for (int o = 0; o < p.noctaves; o++) {
        OctaveParams& q = d->oct[o];
        int s, border1;
        if (o > 0) {
            border1 = ((3 * (mask_size + 4 * octave)) / 2) / (p.sampling * octave) + 1;
            borders[0] = border1;
            borders[1] = border1;
            s = 2;
            for (int t = 0; t < 2; t++) {
                int pl = t == 0 ? p.max_scale - 3 : p.max_scale - 1, oo = o - 1, st = 2;
                while (pl < 2 && oo > 0) {      // a copy of a copy (4 scales per octave)
                    pl = pl == 0 ? p.max_scale - 3 : p.max_scale - 1;
                    oo--;
                    st *= 2;
                }
                q.hbase[t] = d->oct[oo].ooff + (long long)pl * d->oct[oo].osize;
                q.hrow[t] = d->oct[oo].sp * st;
                q.hcol[t] = st;
            }
        } else {
            border1 = ((3 * (mask_size + 6 * octave)) / 2) / (p.sampling * octave) + 1;
            s = 0;
        }
        q.octave = octave;
        q.init_scale = s;
        q.nscale = p.max_scale - s;
        q.delta = p.sampling * octave;
        for (int i = 0, ss = s; ss < p.max_scale; i++, ss++) {
            borders[ss] = border1;
            const int m = mask_size + 2 * octave * (i + 1);
            if (ss > 2) border1 = 3 * m / 2 / q.delta + 1;
            q.mask[i] = m;
            q.b1[i] = border1;
            float nrm = 9.f / (float)(m * m);
            nrm *= nrm;
            q.norm[i] = nrm;
            q.x2[i] = m / 2;
            q.x3[i] = q.x2[i] + q.x2[i];
            q.x4[i] = q.x2[i] + q.x3[i];
            // every box corner inside the integral image (the reference never checks)
            const int reach = std::max(m + q.x2[i], q.x4[i]);
            const int vx = q.sw - 2 * border1, vy = q.sh - 2 * border1;
            if (vx > 0 && vy > 0) {
                if (q.delta * border1 - reach < 0 || q.delta * (q.sw - border1 - 1) + reach + 1 >= iw ||
                    q.delta * (q.sh - border1 - 1) + reach + 1 >= ih)
                    return SURFHIP_ERR_INVALID;
                hbytes += (long long)vx * vy * 4;
            }
        }
        mask_size = q.mask[q.nscale - 1];
        for (int k = 0; k < kMaxScale; k++) q.borders[k] = borders[k];
        int n = 0, maxw = 0, maxh = 0;
        for (int k = 1; k < p.max_scale - 1; k += 2) {
            q.mb[n] = borders[k + 1] + 1;
            const int b = q.mb[n] + q.mb[n];
            maxw = std::max(maxw, q.sw - b);
            maxh = std::max(maxh, q.sh - b);
            n++;
        }
        q.nms_gx = ((maxw / 2 + 16 - 1) / 16) * 16;   // DX = 16, surfd.cu:3060, 3076
        q.nms_gy = ((maxh / 2 + 16 - 1) / 16) * 16;
        octave += octave;
    }
    // compulsory Hessian bytes: the integral image read once + valid responses
    d->hess_bytes = (long long)iw * ih * 4 + hbytes;
    return SURFHIP_OK;
}

static void free_all(surfhip_detector* d)
{
    void* ptrs[] = {d->d_oct, d->iib[0], d->iib[1], d->resp, d->colsum, d->rowseg, d->cand, d->keys, d->gscratch, d->cand_count,
                    d->scan_key, d->scan_src, d->scan_cube, d->item_count, d->item_off,
                    d->offsets, d->order, d->work, d->status, d->pts1, d->desc1, d->count1, d->dbl};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (int i = 0; i < SURFHIP_NSTAGE; i++)
        if (d->ev[i]) (void)hipEventDestroy(d->ev[i]);
    for (int i = 0; i < SURFHIP_MAX_HESS_EV; i++)
        for (int j = 0; j < 3; j++)
            if (d->hev[i][j]) (void)hipEventDestroy(d->hev[i][j]);
    if (d->fork) (void)hipEventDestroy(d->fork);
    if (d->fork2) (void)hipEventDestroy(d->fork2);
    if (d->join) (void)hipEventDestroy(d->join);
    if (d->side) (void)hipStreamDestroy(d->side);
}

int surfhip_detector_create(surfhip_detector** out, const surfhip_param* param, int width, int height,
                            int max_batch, int max_pts, int cand_cap, void* stream)
{
    if (!out || !param || width < 16 || height < 16 || max_batch < 1 || max_pts < 1) return SURFHIP_ERR_INVALID;
    if (width + 1 > 8192) return SURFHIP_ERR_UNSUPPORTED;     // integral kernels: <= 32 columns per thread
    surfhip_param chk;
    int rc = surfhip_make_param(&chk, param->noctaves, param->thresh, param->doubled, param->init_lobe * 3,
                                param->doubled ? param->sampling / 2 : param->sampling, param->upright,
                                param->extend, param->desc_wsz);
    if (rc != SURFHIP_OK) return rc;
    surfhip_detector* d = new surfhip_detector();
    d->param = chk;
    d->srcW = width;
    d->srcH = height;
    // doubled (surf.cpp:234-235, 377-378): the integral is taken of the
    // (2W-2) x (2H-2) upsampled frames D, giving the (2W-1) x (2H-1) grid
    d->W = chk.doubled ? 2 * width - 2 : width;
    d->H = chk.doubled ? 2 * height - 2 : height;
    if (d->W + 1 > 8192) {
        delete d;
        return SURFHIP_ERR_UNSUPPORTED;
    }
    d->max_batch = max_batch;
    d->max_pts = max_pts;
    int cap = cand_cap > 0 ? cand_cap : std::max(max_pts, kSortCap);
    int c2 = 1;
    while (c2 < cap) c2 <<= 1;
    d->cap = c2;
    d->stream = (hipStream_t)stream;
    hipError_t e = hipGetDevice(&d->dev);
    if (e == hipSuccess) {
        hipDeviceProp_t pr;
        e = hipGetDeviceProperties(&pr, d->dev);
        if (e == hipSuccess) d->cus = pr.multiProcessorCount;
    }
    rc = (e == hipSuccess) ? derive(d) : SURFHIP_ERR_HIP;
    // the NMS survivor records pack the sample row / column into 14 bits and
    // the block row of the canonical key into 13 (k_nms_scan): octave 0 is
    // the largest octave, so its extent bounds them all
    if (rc == SURFHIP_OK && (d->oct[0].sh >= 16384 || d->oct[0].sw >= 16384 || d->oct[0].nms_gy >= 8192))
        rc = SURFHIP_ERR_UNSUPPORTED;
    if (rc != SURFHIP_OK) {
        if (e != hipSuccess) g_last_hip = e;
        delete d;
        return rc;
    }
    d->nbands = (d->H + big_band_rows() - 1) / big_band_rows();
    d->CW = (d->W + 1 <= 2048) ? 2048 : (d->W + 1 <= 4096 ? 4096 : 8192);
    const size_t B = (size_t)max_batch;
#define ALLOC(ptr, bytes)                                    \
    do {                                                     \
        e = hipMalloc((void**)&(ptr), (bytes));              \
        if (e != hipSuccess) goto fail;                      \
    } while (0)
    make_plan(d->P, d->oct, d->plan, max_batch);
    if (d->plan.iiw) {
        // the stage also writes the integral image (read: the u8 frame)
        d->hess_bytes += (long long)d->W * d->H;
        ALLOC(d->rowseg, B * d->plan.rs_nstrips * d->plan.rs_rows * sizeof(uint32_t));
    }
    ALLOC(d->d_oct, sizeof(OctaveParams) * kMaxOct);
    ALLOC(d->iib[0], B * d->P.ii_stride * sizeof(int32_t));
    d->ii = d->iib[0];
    ALLOC(d->resp, B * d->tot_osize * sizeof(float));
    ALLOC(d->colsum, (size_t)integral_bands(d->H, B) * d->CW * sizeof(uint32_t));
    ALLOC(d->cand, B * d->cap * sizeof(surfhip_point));
    ALLOC(d->keys, B * d->cap * sizeof(uint32_t));
    ALLOC(d->cand_count, B * sizeof(int));
    d->nitems = d->plan.nms_start[kMaxOct] * 4;
    ALLOC(d->scan_key, B * (size_t)d->nitems * kItemCap * sizeof(uint32_t));
    ALLOC(d->scan_src, B * (size_t)d->nitems * kItemCap * sizeof(uint32_t));
    ALLOC(d->scan_cube, B * (size_t)d->nitems * kCubeCap * kCubeF * sizeof(float));
    ALLOC(d->item_count, B * (size_t)d->nitems * sizeof(int));
    // prefix (nitems + 1) followed by the scan's per-chunk totals
    ALLOC(d->item_off, (2 * B * (size_t)d->nitems + 64) * sizeof(int));
    ALLOC(d->offsets, (B + 1) * sizeof(int));
    ALLOC(d->order, B * (size_t)max_pts * sizeof(int));
    ALLOC(d->work, B * (size_t)max_pts * kWorkF4 * sizeof(float4));
    ALLOC(d->status, 256 + kDescQueueBytes);    // [0]: flags; from [64]: describe work queues
    ALLOC(d->pts1, (size_t)max_pts * sizeof(surfhip_point));
    ALLOC(d->desc1, (size_t)max_pts * d->param.nfeatures * sizeof(float));
    ALLOC(d->count1, 16);
    if (d->cap > kSortCap) ALLOC(d->gscratch, B * d->cap * sizeof(uint64_t));
    if (d->param.doubled) {
        d->dpitch = align_up(d->W, 128);
        d->dstride = (long long)d->H * d->dpitch;
        ALLOC(d->dbl, B * (size_t)d->dstride);
    }
#undef ALLOC
    // zero once: integral pad columns and response pad columns are never
    // written by the kernels and never read by them either
    e = hipMemcpy(d->d_oct, d->oct, sizeof(OctaveParams) * kMaxOct, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(d->iib[0], 0, B * d->P.ii_stride * sizeof(int32_t));
    if (e == hipSuccess) e = hipMemset(d->resp, 0, B * d->tot_osize * sizeof(float));
    if (e == hipSuccess) e = hipMemset(d->status, 0, 16);
    // strip 0's slab and the rows past H stay zero (k_ii_rowseg never writes them)
    if (e == hipSuccess && d->rowseg)
        e = hipMemset(d->rowseg, 0, B * d->plan.rs_nstrips * d->plan.rs_rows * sizeof(uint32_t));
    if (e != hipSuccess) goto fail;
    {
        // LUTs (surf.cpp:358-371) and orientation bins (surf.cpp:83-89); the
        // values are geometry-independent, so one constant table serves all
        Tables t;
        for (int n = 0; n < 83; n++) t.lut1[n] = expf(-(n + 0.5f) / 12.5f);
        for (int n = 0; n < 40; n++) t.lut2[n] = expf(-(n + 0.5f) / 8.f);
        t.bins[0] = (float)(-3.14159265358979323846);
        for (int i = 1; i < 72; i++) t.bins[i] = t.bins[i - 1] + 0.08726646259971647f;
        e = set_tables(t);
        if (e != hipSuccess) goto fail;
    }
    for (int i = 0; i < SURFHIP_NSTAGE; i++) {
        e = hipEventCreate(&d->ev[i]);
        if (e != hipSuccess) goto fail;
    }
    e = hipStreamCreateWithFlags(&d->side, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&d->fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&d->join, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&d->fork2, hipEventDisableTiming);
    if (e != hipSuccess) goto fail;
    *out = d;
    return SURFHIP_OK;
fail:
    g_last_hip = e;
    free_all(d);
    delete d;
    return e == hipErrorOutOfMemory ? SURFHIP_ERR_NOMEM : SURFHIP_ERR_HIP;
}

int surfhip_detector_destroy(surfhip_detector* d)
{
    if (!d) return SURFHIP_ERR_INVALID;
    (void)hipStreamSynchronize(d->stream);
    if (d->side) (void)hipStreamSynchronize(d->side);    // a next-batch integral may still run there
    free_all(d);
    delete d;
    return SURFHIP_OK;
}

int surfhip_detector_set_stream(surfhip_detector* d, void* stream)
{
    if (!d) return SURFHIP_ERR_INVALID;
    d->stream = (hipStream_t)stream;
    return SURFHIP_OK;
}

static int check_frames(surfhip_detector* d, const uint8_t* frames, int nframes, int pitch, size_t stride)
{
    if (!d || !frames || nframes < 1 || nframes > d->max_batch) return SURFHIP_ERR_INVALID;
    if (pitch < d->srcW || (pitch & 15) != 0) return SURFHIP_ERR_INVALID;
    if (((uintptr_t)frames & 15) != 0) return SURFHIP_ERR_INVALID;
    if (nframes > 1 && (stride < (size_t)pitch * d->srcH || (stride & 15) != 0)) return SURFHIP_ERR_INVALID;
    return SURFHIP_OK;
}

// doubled: upsample the caller's frames into d->dbl and continue from there
static hipError_t source_frames(surfhip_detector* d, const uint8_t*& frames, int& pitch, size_t& stride,
                                int nframes, hipStream_t s)
{
    if (!d->param.doubled) return hipSuccess;
    hipError_t e = launch_double(frames, pitch, (long long)stride, nframes, d->srcW, d->srcH, d->dbl, d->dpitch,
                                 d->dstride, s);
    frames = d->dbl;
    pitch = d->dpitch;
    stride = (size_t)d->dstride;
    return e;
}

int surfhip_run_integral(surfhip_detector* d, const uint8_t* frames, int nframes, int pitch, size_t stride)
{
    int rc = check_frames(d, frames, nframes, pitch, stride);
    if (rc) return rc;
    // a prefetch on the side stream may still be using the colsum scratch
    HIPCHK(hipEventRecord(d->join, d->side));
    HIPCHK(hipStreamWaitEvent(d->stream, d->join, 0));
    HIPCHK(source_frames(d, frames, pitch, stride, nframes, d->stream));
    HIPCHK(launch_integral(frames, pitch, (long long)stride, nframes, d->P, d->colsum, d->ii, d->stream));
    // (plan.iiw) the row sums a following run_hessian's k_hess_w adds: it
    // rewrites the same integral image
    HIPCHK(launch_rowseg(frames, pitch, (long long)stride, nframes, d->P, d->plan, d->rowseg, d->stream));
    d->pref_valid = false;
    d->last_frames = frames;
    d->last_pitch = pitch;
    d->last_fstride = (long long)stride;
    return SURFHIP_OK;
}

int surfhip_run_hessian(surfhip_detector* d, int nframes)
{
    if (!d || nframes < 1 || nframes > d->max_batch) return SURFHIP_ERR_INVALID;
    // the u8 Hessian kernels read the frames of the last run_integral
    if (!d->last_frames && plan_reads_frames(d->plan)) return SURFHIP_ERR_INVALID;
    HIPCHK(launch_hessian(d->last_frames, d->last_pitch, d->last_fstride, d->ii, d->resp, nframes, d->P, d->d_oct,
                          d->oct, d->plan, d->stream, 3, d->rowseg, d->ii));
    return SURFHIP_OK;
}

// The second integral buffer is allocated on first use of the pipelined
// entry point (a plain detect_batch caller never pays for it).
static hipError_t ensure_second_ii(surfhip_detector* d)
{
    if (d->iib[1]) return hipSuccess;
    const size_t bytes = (size_t)d->max_batch * d->P.ii_stride * sizeof(int32_t);
    hipError_t e = hipMalloc((void**)&d->iib[1], bytes);
    if (e == hipSuccess) e = hipMemset(d->iib[1], 0, bytes);     // pad columns stay 0
    return e;
}

int surfhip_detect_batch_next(surfhip_detector* d, const uint8_t* frames, int nframes, int pitch, size_t stride,
                              surfhip_point* points, float* desc, int* counts, const uint8_t* next_frames,
                              int next_nframes, int next_pitch, size_t next_stride)
{
    int rc = check_frames(d, frames, nframes, pitch, stride);
    if (rc) return rc;
    if (!points || !counts) return SURFHIP_ERR_INVALID;
    // no prefetch for doubled frames (the upsampled frames share one scratch
    // buffer) or while stage profiling (serial stages)
    const bool pipe = next_frames != nullptr && !d->param.doubled && !d->profiling;
    if (next_frames && !d->param.doubled) {
        rc = check_frames(d, next_frames, next_nframes, next_pitch, next_stride);
        if (rc) return rc;
    }
    // (plan.iiw: the integral is written by this batch's Hessian, one buffer)
    const bool iiw = d->plan.iiw != 0;
    if (pipe && !iiw) HIPCHK(ensure_second_ii(d));
    hipStream_t s = d->stream;
    const bool prof = d->profiling;
    // this batch's integral (iiw: its row sums): prefetched by the previous
    // call (same frames), or computed now
    const bool have = !prof && d->pref_valid && d->pref_frames == frames && d->pref_n == nframes &&
                      d->pref_pitch == pitch && d->pref_stride == stride;
    d->icur = (have && !iiw) ? d->ipref : (iiw ? 0 : d->icur);
    d->ii = d->iib[d->icur];
    d->pref_valid = false;
    // (the per-batch counters -- accepted candidates per frame, the
    // truncation flag, the scan items' survivor counts -- are written by the
    // NMS scan itself: no memsets ahead of the Hessian)
    if (prof) {
        // serial, so that the stage events bracket each stage alone; a
        // prefetch left on the side stream by an earlier pipelined call may
        // still be using the colsum scratch the integral below reuses
        HIPCHK(hipEventRecord(d->join, d->side));
        HIPCHK(hipStreamWaitEvent(s, d->join, 0));
        HIPCHK(hipEventRecord(d->ev[0], s));
        HIPCHK(source_frames(d, frames, pitch, stride, nframes, s));
        if (iiw) HIPCHK(launch_rowseg(frames, pitch, (long long)stride, nframes, d->P, d->plan, d->rowseg, s));
        else HIPCHK(launch_integral(frames, pitch, (long long)stride, nframes, d->P, d->colsum, d->ii, s));
        HIPCHK(hipEventRecord(d->ev[1], s));
        HIPCHK(launch_hessian(frames, pitch, (long long)stride, d->ii, d->resp, nframes, d->P, d->d_oct, d->oct,
                              d->plan, s, 3, d->rowseg, d->ii));
        HIPCHK(hipEventRecord(d->ev[2], s));
    } else {
        // In-step Hessian timing brackets the WHOLE stage: from the fork (on
        // s) to the end of the u8 kernels on s and of the integral-image
        // kernels on the side stream, whichever is later
        // (surfhip_detector_hessian_times).  Without a prefetched integral
        // the side stream's part starts after the integral, which the
        // bracket then includes.
        HIPCHK(source_frames(d, frames, pitch, stride, nframes, s));
        const bool th = d->time_hess && d->hev_n < SURFHIP_MAX_HESS_EV;
        if (iiw) {
            // octaves 0-3 on the u8 kernels, the integral image written by
            // k_hess_w, any later octave's k_hessian after them (it reads
            // that integral): one stream.  The side stream's last work (a
            // prefetch of d->rowseg) is ordered before the row sums' use:
            // before this call's own row-sum pass, or, prefetched, between
            // the octave-0 kernel and k_hess_w, where the wait's latency
            // hides behind the running octave-0 kernel (iiw 2: the octave-0
            // kernel writes the integral, so the wait precedes it).
            const bool p0w = d->plan.iiw == 2;
            HIPCHK(hipEventRecord(d->join, d->side));
            if (!have || p0w) HIPCHK(hipStreamWaitEvent(s, d->join, 0));
            if (!have)
                HIPCHK(launch_rowseg(frames, pitch, (long long)stride, nframes, d->P, d->plan, d->rowseg, s));
            if (th) HIPCHK(hipEventRecord(d->hev[d->hev_n][0], s));
            HIPCHK(launch_hessian(frames, pitch, (long long)stride, d->ii, d->resp, nframes, d->P, d->d_oct, d->oct,
                                  d->plan, s, 4, d->rowseg, d->ii));
            if (have && !p0w) HIPCHK(hipStreamWaitEvent(s, d->join, 0));
            HIPCHK(launch_hessian(frames, pitch, (long long)stride, d->ii, d->resp, nframes, d->P, d->d_oct, d->oct,
                                  d->plan, s, 8 | 2, d->rowseg, d->ii));
            if (th) {
                HIPCHK(hipEventRecord(d->hev[d->hev_n][1], s));
                d->hev_side[d->hev_n++] = false;
            }
        } else {
        if (th) HIPCHK(hipEventRecord(d->hev[d->hev_n][0], s));
        if (!plan_reads_frames(d->plan)) {
            // Every Hessian kernel reads the integral image (the gather plan
            // of batches <= kGatherBatch, config #2): nothing would run beside
            // them, so they stay on the detector stream -- the fork / join
            // round trip through the side stream cost a one-frame step ~30 us
            // of idle GPU in a kernel trace (profiles/r05ac2_*).  The side
            // stream's last work (a prefetch into d->ii, or one using the
            // colsum scratch) is ordered first; it finished long ago.
            HIPCHK(hipEventRecord(d->join, d->side));
            HIPCHK(hipStreamWaitEvent(s, d->join, 0));
            if (!have)
                HIPCHK(launch_integral(frames, pitch, (long long)stride, nframes, d->P, d->colsum, d->ii, s));
            HIPCHK(launch_hessian(frames, pitch, (long long)stride, d->ii, d->resp, nframes, d->P, d->d_oct,
                                  d->oct, d->plan, s, 2));
            if (th) {
                HIPCHK(hipEventRecord(d->hev[d->hev_n][1], s));
                d->hev_side[d->hev_n++] = false;
            }
        } else {
            // the u8 Hessian kernels need no integral image: they run on s;
            // the integral (unless prefetched) and the integral-image Hessian
            // kernels run on the side stream beside them; s waits for both
            // before NMS
            const bool side_hess = d->plan.hess_start[kMaxOct] > 0;
            HIPCHK(hipEventRecord(d->fork, s));
            HIPCHK(hipStreamWaitEvent(d->side, d->fork, 0));
            if (!have)
                HIPCHK(launch_integral(frames, pitch, (long long)stride, nframes, d->P, d->colsum, d->ii, d->side));
            HIPCHK(launch_hessian(frames, pitch, (long long)stride, d->ii, d->resp, nframes, d->P, d->d_oct,
                                  d->oct, d->plan, d->side, 2));
            if (th && side_hess) HIPCHK(hipEventRecord(d->hev[d->hev_n][2], d->side));
            HIPCHK(hipEventRecord(d->join, d->side));
            HIPCHK(launch_hessian(frames, pitch, (long long)stride, d->ii, d->resp, nframes, d->P, d->d_oct,
                                  d->oct, d->plan, s, 1));
            if (th) {
                HIPCHK(hipEventRecord(d->hev[d->hev_n][1], s));
                d->hev_side[d->hev_n++] = side_hess;
            }
            HIPCHK(hipStreamWaitEvent(s, d->join, 0));
        }
        }
    }
    // The next batch's integral (into the other buffer) on the side stream,
    // ordered after everything on s so far, so that buffer's last readers
    // (the previous batch's fit and describe) are done.  Default: forked
    // after this batch's Hessian, beside its NMS scan, fit and sort (the
    // Hessian and describe then run alone); SURFHIP_PREFETCH=describe forks
    // it after the sort instead, beside describe.  With the integral written
    // by k_hess_w (iiw) the prefetch is only the row-sum pass and the default
    // is beside describe (its HBM use is low and its waves leave room).
    auto prefetch_next = [&]() -> hipError_t {
        const int nx = d->icur ^ 1;
        hipError_t e = hipEventRecord(d->fork2, s);
        if (e == hipSuccess) e = hipStreamWaitEvent(d->side, d->fork2, 0);
        // (iiw: the next batch's row sums; this batch's k_hess_w has read d->rowseg)
        if (e == hipSuccess && iiw)
            e = launch_rowseg(next_frames, next_pitch, (long long)next_stride, next_nframes, d->P, d->plan,
                              d->rowseg, d->side);
        else if (e == hipSuccess)
            e = launch_integral(next_frames, next_pitch, (long long)next_stride, next_nframes, d->P, d->colsum,
                                d->iib[nx], d->side);
        if (e != hipSuccess) return e;
        d->pref_valid = true;
        d->ipref = nx;
        d->pref_frames = next_frames;
        d->pref_n = next_nframes;
        d->pref_pitch = next_pitch;
        d->pref_stride = next_stride;
        return hipSuccess;
    };
    // (iiw: the prefetch is the row-sum pass, default beside describe, whose
    // waves leave room for its 16-VGPR waves; SURFHIP_PREFETCH=nms / describe)
    static const int pref_env = [] {
        const char* e = getenv("SURFHIP_PREFETCH");
        return !e ? -1 : !strcmp(e, "describe") ? 0 : 1;
    }();
    const bool pref_nms = pref_env < 0 ? !iiw : pref_env == 1;
    if (pipe && pref_nms) HIPCHK(prefetch_next());
    // getTrace in k_describe_u2 (its integral rows are in L2 there) rather
    // than in the fit (16 scattered integral loads per survivor from HBM)
    const bool trace_desc = desc && trace_in_describe(d->P, nframes);
    HIPCHK(launch_nms(d->ii, d->resp, nframes, d->P, d->d_oct, d->plan, d->scan_key, d->scan_src, d->scan_cube,
                      d->item_count, d->item_off, d->cand, d->keys, d->cand_count, d->cap, d->status, s, trace_desc));
    if (prof) HIPCHK(hipEventRecord(d->ev[3], s));
    HIPCHK(launch_sort(d->cand, d->keys, d->gscratch, d->cand_count, d->item_off, d->plan.nms_start[kMaxOct] * 4,
                       d->cap, nframes, points, d->max_pts, counts, d->offsets, d->order, d->status, s));
    if (prof) HIPCHK(hipEventRecord(d->ev[4], s));
    if (pipe && !pref_nms) HIPCHK(prefetch_next());
    if (d->desc_ev) HIPCHK(hipEventRecord(d->desc_ev, s));
    if (desc)
        HIPCHK(launch_describe(d->ii, d->P, points, d->max_pts, counts, d->offsets, d->order, d->work, nframes, desc,
                               d->status + 64, s, pipe && !pref_nms && !iiw, d->cus, trace_desc));
    if (prof) HIPCHK(hipEventRecord(d->ev[5], s));
    d->last_nframes = nframes;
    d->last_frames = frames;
    d->last_pitch = pitch;
    d->last_fstride = (long long)stride;
    return SURFHIP_OK;
}

int surfhip_detector_set_describe_event(surfhip_detector* d, void* ev)
{
    if (!d) return SURFHIP_ERR_INVALID;
    d->desc_ev = (hipEvent_t)ev;
    return SURFHIP_OK;
}

int surfhip_detector_drain(surfhip_detector* d)
{
    if (!d) return SURFHIP_ERR_INVALID;
    // everything queued on the side stream so far (a prefetch of the next
    // batch's integral, which reads next_frames) is ordered before the
    // detector stream's later work
    HIPCHK(hipEventRecord(d->join, d->side));
    HIPCHK(hipStreamWaitEvent(d->stream, d->join, 0));
    return SURFHIP_OK;
}

int surfhip_detect_batch(surfhip_detector* d, const uint8_t* frames, int nframes, int pitch,
                         size_t stride, surfhip_point* points, float* desc, int* counts)
{
    return surfhip_detect_batch_next(d, frames, nframes, pitch, stride, points, desc, counts, nullptr, 0, 0, 0);
}

int surfhip_detect(surfhip_detector* d, const uint8_t* image, int pitch, surfhip_point* points,
                   int max_pts, int* num_pts, float** desc_out, int desc)
{
    if (!d || !points || !num_pts || max_pts < 0) return SURFHIP_ERR_INVALID;
    int rc = surfhip_detect_batch(d, image, 1, pitch, 0, d->pts1, desc ? d->desc1 : nullptr, d->count1);
    if (rc) return rc;
    // A frame with more candidates than the detector's capacity keeps the
    // first `cap` NMS survivors in scan order (deterministic) and returns
    // them like any other frame, as the reference returns max_pts points
    // (surf.cpp:302-303); surfhip_detector_status() tells the caller.
    int cnt = 0;
    HIPCHK(hipMemcpyAsync(&cnt, d->count1, sizeof(int), hipMemcpyDeviceToHost, d->stream));
    HIPCHK(hipStreamSynchronize(d->stream));
    const int n = std::min(cnt, max_pts);                  // surf.cpp:303
    if (n > 0)
        HIPCHK(hipMemcpyAsync(points, d->pts1, sizeof(surfhip_point) * n, hipMemcpyDeviceToDevice, d->stream));
    if (desc && desc_out) {
        const size_t nb = sizeof(float) * (size_t)std::max(n, 1) * d->param.nfeatures;
        HIPCHK(hipMalloc((void**)desc_out, nb));                // cuDescribe's per-call cudaMalloc, surfd.cu:3264
        if (n > 0)
            HIPCHK(hipMemcpyAsync(*desc_out, d->desc1, sizeof(float) * (size_t)n * d->param.nfeatures,
                                  hipMemcpyDeviceToDevice, d->stream));
    }
    HIPCHK(hipStreamSynchronize(d->stream));
    *num_pts = n;
    return SURFHIP_OK;
}

int surfhip_detector_candidates(surfhip_detector* d, int* h_counts, int nframes)
{
    if (!d || !h_counts || nframes < 1 || nframes > d->max_batch) return SURFHIP_ERR_INVALID;
    HIPCHK(hipMemcpyAsync(h_counts, d->cand_count, sizeof(int) * nframes, hipMemcpyDeviceToHost, d->stream));
    HIPCHK(hipStreamSynchronize(d->stream));
    int st = 0;
    HIPCHK(hipMemcpy(&st, d->status, sizeof(int), hipMemcpyDeviceToHost));
    return st ? SURFHIP_ERR_CAPACITY : SURFHIP_OK;
}

int surfhip_detector_status(surfhip_detector* d, int* truncated)
{
    if (!d || !truncated) return SURFHIP_ERR_INVALID;
    int st = 0;
    HIPCHK(hipMemcpyAsync(&st, d->status, sizeof(int), hipMemcpyDeviceToHost, d->stream));
    HIPCHK(hipStreamSynchronize(d->stream));
    *truncated = st & 1;
    return SURFHIP_OK;
}

int surfhip_detector_capacity(surfhip_detector* d, int* cand_cap)
{
    if (!d || !cand_cap) return SURFHIP_ERR_INVALID;
    *cand_cap = d->cap;
    return SURFHIP_OK;
}

int surfhip_detector_set_profiling(surfhip_detector* d, int on)
{
    if (!d) return SURFHIP_ERR_INVALID;
    d->profiling = on != 0;
    return SURFHIP_OK;
}

int surfhip_detector_stage_times(surfhip_detector* d, float* ms)
{
    if (!d || !ms || !d->profiling) return SURFHIP_ERR_INVALID;
    HIPCHK(hipEventSynchronize(d->ev[SURFHIP_NSTAGE - 1]));
    for (int i = 0; i < SURFHIP_NSTAGE - 1; i++) HIPCHK(hipEventElapsedTime(&ms[i], d->ev[i], d->ev[i + 1]));
    HIPCHK(hipEventElapsedTime(&ms[SURFHIP_NSTAGE - 1], d->ev[0], d->ev[SURFHIP_NSTAGE - 1]));
    return SURFHIP_OK;
}

int surfhip_detector_time_hessian(surfhip_detector* d, int on)
{
    if (!d) return SURFHIP_ERR_INVALID;
    if (on) {
        for (int i = 0; i < SURFHIP_MAX_HESS_EV; i++)
            for (int j = 0; j < 3; j++)
                if (!d->hev[i][j]) HIPCHK(hipEventCreate(&d->hev[i][j]));
    }
    d->time_hess = on != 0;
    d->hev_n = 0;
    return SURFHIP_OK;
}

int surfhip_detector_hessian_times(surfhip_detector* d, float* ms, int max, int* n)
{
    if (!d || !n || (max > 0 && !ms)) return SURFHIP_ERR_INVALID;
    const int k = std::min(d->hev_n, std::max(max, 0));
    for (int i = 0; i < k; i++) {
        HIPCHK(hipEventSynchronize(d->hev[i][1]));
        HIPCHK(hipEventElapsedTime(&ms[i], d->hev[i][0], d->hev[i][1]));
        if (d->hev_side[i]) {
            float t2 = 0.f;
            HIPCHK(hipEventSynchronize(d->hev[i][2]));
            HIPCHK(hipEventElapsedTime(&t2, d->hev[i][0], d->hev[i][2]));
            ms[i] = std::max(ms[i], t2);
        }
    }
    *n = k;
    d->hev_n = 0;
    return SURFHIP_OK;
}

int surfhip_detector_workspace(surfhip_detector* d, int32_t** ii, size_t* ii_stride, float** resp,
                               size_t* resp_stride)
{
    if (!d) return SURFHIP_ERR_INVALID;
    if (ii) *ii = d->ii;
    if (ii_stride) *ii_stride = (size_t)d->P.ii_stride;
    if (resp) *resp = d->resp;
    if (resp_stride) *resp_stride = (size_t)d->P.resp_stride;
    return SURFHIP_OK;
}

int surfhip_detector_geometry(surfhip_detector* d, int* iwhp, int* swhp, long long* ooff, int* osize)
{
    if (!d) return SURFHIP_ERR_INVALID;
    if (iwhp) { iwhp[0] = d->W + 1; iwhp[1] = d->H + 1; iwhp[2] = d->P.ip; }
    for (int o = 0; o < kMaxOct; o++) {
        const bool v = o < d->param.noctaves;
        if (swhp) { swhp[3 * o] = v ? d->oct[o].sw : 0; swhp[3 * o + 1] = v ? d->oct[o].sh : 0; swhp[3 * o + 2] = v ? d->oct[o].sp : 0; }
        if (ooff) ooff[o] = v ? d->oct[o].ooff : 0;
        if (osize) osize[o] = v ? d->oct[o].osize : 0;
    }
    return SURFHIP_OK;
}

long long surfhip_hessian_bytes_per_frame(surfhip_detector* d) { return d ? d->hess_bytes : -1; }

int surfhip_hessian_plan(surfhip_detector* d, char* buf, int len)
{
    if (!d) return SURFHIP_ERR_INVALID;
    const std::string t = hessian_plan_text(d->plan, d->P);
    if (buf && len > 0) {
        const size_t n = std::min((size_t)len - 1, t.size());
        memcpy(buf, t.data(), n);
        buf[n] = 0;
    }
    return (int)t.size();
}

size_t surfhip_slab_bytes(int nframes, int total, int nfeatures)
{
    return 16 + (((size_t)nframes * 4 + 15) & ~(size_t)15) +
           (size_t)total * (sizeof(surfhip_point) + sizeof(float) * (size_t)nfeatures);
}

int surfhip_batch_total(surfhip_detector* d, int nframes, int* total)
{
    if (!d || !total || nframes < 1 || nframes > d->max_batch) return SURFHIP_ERR_INVALID;
    HIPCHK(hipMemcpyAsync(total, d->offsets + nframes, sizeof(int), hipMemcpyDeviceToHost, d->stream));
    HIPCHK(hipStreamSynchronize(d->stream));
    return SURFHIP_OK;
}

int surfhip_pack_slab_cap(surfhip_detector* d, const surfhip_point* pts, const float* desc, const int* counts,
                          int nframes, void* slab, size_t cap_bytes)
{
    if (!d || !pts || !counts || !slab || nframes < 1 || nframes > d->max_batch) return SURFHIP_ERR_INVALID;
    if (cap_bytes < surfhip_slab_bytes(nframes, 0, 0)) return SURFHIP_ERR_INVALID;
    HIPCHK(launch_pack(pts, desc, counts, d->offsets, nframes, d->max_pts, d->param.nfeatures, d->status, cap_bytes,
                       (uint8_t*)slab, d->stream));
    return SURFHIP_OK;
}

int surfhip_pack_slab(surfhip_detector* d, const surfhip_point* pts, const float* desc, const int* counts,
                      int nframes, void* slab)
{
    return surfhip_pack_slab_cap(d, pts, desc, counts, nframes, slab, (size_t)-1);
}

size_t surfhip_match_scratch(int n1, int n2, int flags)
{
    if (n1 < 0 || n2 < 0) return 0;
    return match_scratch_bytes(n1, n2, flags);
}

int surfhip_match(surfhip_point* pts1, const surfhip_point* pts2, const float* f1, const float* f2, int n1, int n2,
                  int nf, int flags, void* scratch, void* stream)
{
    if (n1 < 0 || n2 < 0 || nf < 4 || nf > 1024 || (nf & 3) || (flags & ~SURFHIP_MATCH_FULL_TAIL))
        return SURFHIP_ERR_INVALID;
    if (n1 == 0) return SURFHIP_OK;
    if (!pts1 || !f1 || (n2 > 0 && (!pts2 || !f2))) return SURFHIP_ERR_INVALID;
    hipStream_t s = (hipStream_t)stream;
    const size_t bytes = match_scratch_bytes(n1, n2, flags);
    void* own = nullptr;
    if (!scratch && bytes) {            // no caller scratch: allocate, and finish before freeing it
        HIPCHK(hipMalloc(&own, bytes));
        scratch = own;
    }
    hipError_t e = launch_match(pts1, pts2, f1, f2, n1, n2, nf, flags, scratch, s);
    if (own) {
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        hipError_t e2 = hipFree(own);
        if (e == hipSuccess) e = e2;
    }
    HIPCHK(e);
    return SURFHIP_OK;
}

/* ------------------------------------------------------------- ingest --
 * Pipelined host -> HBM -> result-slab ring.  The
 * reference feeds one frame per call through a blocking cudaMemcpy2D of a
 * pageable OpenCV buffer (main.cpp:212-226) and copies each frame's points
 * back with a blocking cudaMemcpy (surf.cpp:335-342).  Here `depth` pinned
 * host frame slots feed `depth` HBM frame slots over a copy stream; the
 * detector stream waits only on its own slot's copy event, so batch i+1's
 * PCIe transfer runs under batch i's kernels.  Each batch is packed into its
 * slot's device slab right after describe (before the next batch may reuse
 * the detector's scratch) and its 16-B header + counts come back
 * asynchronously; collect() then copies exactly the slab's bytes to pinned
 * host memory on a third stream while later batches keep computing. */
struct surfhip_ingest {
    surfhip_detector* det = nullptr;
    int depth = 0, pitch = 0, hdr_bytes = 0;
    size_t frame_bytes = 0, dslab_cap = 0;
    hipStream_t copy = nullptr, out = nullptr;
    uint8_t* h_frames[SURFHIP_INGEST_MAX_DEPTH]{};
    uint8_t* d_frames[SURFHIP_INGEST_MAX_DEPTH]{};
    uint8_t* d_slab[SURFHIP_INGEST_MAX_DEPTH]{};
    int32_t* h_hdr[SURFHIP_INGEST_MAX_DEPTH]{};
    uint8_t* h_slab[SURFHIP_INGEST_MAX_DEPTH]{};
    size_t h_slab_cap[SURFHIP_INGEST_MAX_DEPTH]{};
    int nframes[SURFHIP_INGEST_MAX_DEPTH]{};
    hipEvent_t ev_h2d[SURFHIP_INGEST_MAX_DEPTH]{}, ev_done[SURFHIP_INGEST_MAX_DEPTH]{};
    surfhip_point* d_pts = nullptr;
    float* d_desc = nullptr;
    int* d_counts = nullptr;
    long long submitted = 0, collected = 0;
    int acquired = -1;                  // slot handed out by acquire, not yet submitted
};

static void ingest_free(surfhip_ingest* g)
{
    for (int s = 0; s < SURFHIP_INGEST_MAX_DEPTH; ++s) {
        if (g->h_frames[s]) (void)hipHostFree(g->h_frames[s]);
        if (g->h_hdr[s]) (void)hipHostFree(g->h_hdr[s]);
        if (g->h_slab[s]) (void)hipHostFree(g->h_slab[s]);
        if (g->d_frames[s]) (void)hipFree(g->d_frames[s]);
        if (g->d_slab[s]) (void)hipFree(g->d_slab[s]);
        if (g->ev_h2d[s]) (void)hipEventDestroy(g->ev_h2d[s]);
        if (g->ev_done[s]) (void)hipEventDestroy(g->ev_done[s]);
    }
    if (g->d_pts) (void)hipFree(g->d_pts);
    if (g->d_desc) (void)hipFree(g->d_desc);
    if (g->d_counts) (void)hipFree(g->d_counts);
    if (g->copy) (void)hipStreamDestroy(g->copy);
    if (g->out) (void)hipStreamDestroy(g->out);
    delete g;
}

static int ingest_alloc(surfhip_ingest* g)
{
    surfhip_detector* d = g->det;
    const int nf = d->param.nfeatures, B = d->max_batch;
    g->pitch = (d->srcW + 127) & ~127;
    g->frame_bytes = (size_t)g->pitch * d->srcH;
    g->hdr_bytes = 16 + ((4 * B + 15) & ~15);
    g->dslab_cap = surfhip_slab_bytes(B, B * d->max_pts, nf);
    HIPCHK(hipStreamCreateWithFlags(&g->copy, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&g->out, hipStreamNonBlocking));
    HIPCHK(hipMalloc(&g->d_pts, sizeof(surfhip_point) * (size_t)B * d->max_pts));
    if (nf) HIPCHK(hipMalloc(&g->d_desc, sizeof(float) * (size_t)B * d->max_pts * nf));
    HIPCHK(hipMalloc(&g->d_counts, sizeof(int) * (size_t)B));
    for (int s = 0; s < g->depth; ++s) {
        HIPCHK(hipHostMalloc(&g->h_frames[s], g->frame_bytes * B, hipHostMallocDefault));
        HIPCHK(hipHostMalloc(&g->h_hdr[s], g->hdr_bytes, hipHostMallocDefault));
        HIPCHK(hipMalloc(&g->d_frames[s], g->frame_bytes * B));
        HIPCHK(hipMalloc(&g->d_slab[s], g->dslab_cap));
        HIPCHK(hipEventCreateWithFlags(&g->ev_h2d[s], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&g->ev_done[s], hipEventDisableTiming));
        memset(g->h_frames[s], 0, g->frame_bytes * B);
    }
    return SURFHIP_OK;
}

int surfhip_ingest_create(surfhip_ingest** out, surfhip_detector* det, int depth)
{
    if (!out || !det || depth < 1 || depth > SURFHIP_INGEST_MAX_DEPTH) return SURFHIP_ERR_INVALID;
    *out = nullptr;
    surfhip_ingest* g = new surfhip_ingest;
    g->det = det;
    g->depth = depth;
    int rc = ingest_alloc(g);
    if (rc != SURFHIP_OK) {
        ingest_free(g);
        return rc;
    }
    *out = g;
    return SURFHIP_OK;
}

int surfhip_ingest_destroy(surfhip_ingest* g)
{
    if (!g) return SURFHIP_ERR_INVALID;
    // wait on the ring's own events only: the detector may already be gone
    hipError_t e = hipStreamSynchronize(g->copy);
    for (long long b = g->collected; b < g->submitted; ++b) {
        hipError_t e1 = hipEventSynchronize(g->ev_done[b % g->depth]);
        if (e == hipSuccess) e = e1;
    }
    hipError_t e2 = hipStreamSynchronize(g->out);
    ingest_free(g);
    HIPCHK(e);
    HIPCHK(e2);
    return SURFHIP_OK;
}

int surfhip_ingest_acquire(surfhip_ingest* g, uint8_t** h_frames, int* pitch, size_t* frame_stride)
{
    if (!g || !h_frames) return SURFHIP_ERR_INVALID;
    if (g->submitted - g->collected >= g->depth) return SURFHIP_ERR_CAPACITY;   // collect first
    const int s = (int)(g->submitted % g->depth);
    // the slot's previous batch was collected, so its copy and kernels are done
    g->acquired = s;
    *h_frames = g->h_frames[s];
    if (pitch) *pitch = g->pitch;
    if (frame_stride) *frame_stride = g->frame_bytes;
    return SURFHIP_OK;
}

int surfhip_ingest_submit(surfhip_ingest* g, int nframes)
{
    if (!g || g->acquired < 0 || nframes < 1 || nframes > g->det->max_batch) return SURFHIP_ERR_INVALID;
    surfhip_detector* d = g->det;
    const int s = g->acquired;
    g->acquired = -1;
    g->nframes[s] = nframes;
    HIPCHK(hipMemcpyAsync(g->d_frames[s], g->h_frames[s], g->frame_bytes * nframes, hipMemcpyHostToDevice,
                          g->copy));
    HIPCHK(hipEventRecord(g->ev_h2d[s], g->copy));
    HIPCHK(hipStreamWaitEvent(d->stream, g->ev_h2d[s], 0));
    int rc = surfhip_detect_batch(d, g->d_frames[s], nframes, g->pitch, g->frame_bytes, g->d_pts, g->d_desc,
                                  g->d_counts);
    if (rc != SURFHIP_OK) return rc;
    rc = surfhip_pack_slab(d, g->d_pts, g->d_desc, g->d_counts, nframes, g->d_slab[s]);
    if (rc != SURFHIP_OK) return rc;
    HIPCHK(hipMemcpyAsync(g->h_hdr[s], g->d_slab[s], 16 + ((4 * nframes + 15) & ~15), hipMemcpyDeviceToHost,
                          d->stream));
    HIPCHK(hipEventRecord(g->ev_done[s], d->stream));
    ++g->submitted;
    return SURFHIP_OK;
}

int surfhip_ingest_collect(surfhip_ingest* g, const void** h_slab, size_t* bytes)
{
    if (!g || !h_slab || !bytes) return SURFHIP_ERR_INVALID;
    if (g->collected >= g->submitted) return SURFHIP_ERR_INVALID;        // nothing in flight
    const int s = (int)(g->collected % g->depth);
    HIPCHK(hipEventSynchronize(g->ev_done[s]));
    const int32_t* hdr = g->h_hdr[s];
    if (hdr[0] != g->nframes[s] || hdr[1] < 0) return SURFHIP_ERR_HIP;
    const size_t n = surfhip_slab_bytes(hdr[0], hdr[1], hdr[2]);
    if (n > g->h_slab_cap[s]) {
        if (g->h_slab[s]) HIPCHK(hipHostFree(g->h_slab[s]));
        g->h_slab[s] = nullptr;
        g->h_slab_cap[s] = 0;
        const size_t cap = n + n / 4;
        HIPCHK(hipHostMalloc(&g->h_slab[s], cap, hipHostMallocDefault));
        g->h_slab_cap[s] = cap;
    }
    HIPCHK(hipMemcpyAsync(g->h_slab[s], g->d_slab[s], n, hipMemcpyDeviceToHost, g->out));
    HIPCHK(hipStreamSynchronize(g->out));
    ++g->collected;
    *h_slab = g->h_slab[s];
    *bytes = n;
    return SURFHIP_OK;
}

int surfhip_ingest_pending(surfhip_ingest* g, int* n)
{
    if (!g || !n) return SURFHIP_ERR_INVALID;
    *n = (int)(g->submitted - g->collected);
    return SURFHIP_OK;
}

/* --------------------------------------------------------------- dump --
 * Keypoint + descriptor file: a sequence of records, each a 64-B header
 * followed by one result slab (the all-gather format above).  The reference
 * has no on-disk format (it only draws keypoints, main.cpp:21-71). */
int surfhip_dump_append(const char* path, const void* h_slab, size_t bytes, int width, int height,
                        const surfhip_param* p, long long first_frame)
{
    if (!path || !h_slab || bytes < 16 || !p) return SURFHIP_ERR_INVALID;
    const int32_t* sh = (const int32_t*)h_slab;
    if (sh[0] < 0 || sh[1] < 0 || surfhip_slab_bytes(sh[0], sh[1], sh[2]) != bytes) return SURFHIP_ERR_INVALID;
    surfhip_dump_header h;
    memset(&h, 0, sizeof h);
    memcpy(h.magic, SURFHIP_DUMP_MAGIC, 8);
    h.header_bytes = sizeof h;
    h.version = SURFHIP_DUMP_VERSION;
    h.width = (uint32_t)width;
    h.height = (uint32_t)height;
    h.nframes = (uint32_t)sh[0];
    h.nfeatures = (uint32_t)sh[2];
    h.total = (uint64_t)sh[1];
    h.slab_bytes = (uint64_t)bytes;
    h.first_frame = (uint64_t)first_frame;
    h.thresh = p->thresh;
    h.noctaves = (uint8_t)p->noctaves;
    h.upright = p->upright ? 1 : 0;
    h.extend = p->extend ? 1 : 0;
    h.doubled = p->doubled ? 1 : 0;
    FILE* f = fopen(path, "ab");
    if (!f) return SURFHIP_ERR_INVALID;
    int ok = fwrite(&h, sizeof h, 1, f) == 1 && fwrite(h_slab, 1, bytes, f) == bytes;
    ok = (fclose(f) == 0) && ok;
    return ok ? SURFHIP_OK : SURFHIP_ERR_INVALID;
}

int surfhip_stream_run(int mode, const void* src, void* dst, size_t bytes, void* stream)
{
    if (mode < 0 || mode > 2 || bytes % 16 != 0 || ((uintptr_t)src & 15) || ((uintptr_t)dst & 15) ||
        (mode != 2 && !src) || (mode != 1 && !dst))
        return SURFHIP_ERR_INVALID;
    if (bytes == 0) return SURFHIP_OK;
    int dev = 0, ncu = 0;
    HIPCHK(hipGetDevice(&dev));
    HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    HIPCHK(surfhip::launch_stream(mode, src, dst, bytes, ncu, (hipStream_t)stream));
    return SURFHIP_OK;
}

size_t surfhip_stream_bytes(int mode, size_t bytes) { return mode == 0 ? 2 * bytes : mode == 1 || mode == 2 ? bytes : 0; }

const char* surfhip_build_info(void)
{
    return "libsurfhip gfx950 (" __DATE__ " " __TIME__ ")";
}

}  // extern "C"
