// surfhip_internal.h -- parameter blocks and launch helpers shared by the
// kernel TU (surfhip_kernels.hip) and the C-ABI TU (surfhip_api.hip).
//
// The reference keeps these values in process-global __constant__ symbols
// that every frame re-uploads (surfd.cu:13-24, 27-102; 22 cudaMemcpyToSymbol
// per frame at 4 octaves).  Here they are computed once per detector and
// passed by value as kernel arguments, so detectors are independent and a
// frame costs no host->device parameter traffic.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <string>

#include "surfhip.h"

namespace surfhip {

constexpr int kMaxOct = 8;
constexpr int kMaxScale = 8;
constexpr int kSortCap = 16384;     // candidates per frame sorted in LDS
constexpr uint32_t kNoKey = 0xffffffffu;   // candidate slot of a rejected NMS survivor
#ifndef SURF_DESC_Q
#define SURF_DESC_Q 16                      // (A/B: <= 16; the queue memset covers 16)
#endif
constexpr int kDescQ = SURF_DESC_Q;         // describe work queues per XCD
constexpr int kDescQueueBytes = 8 * kDescQ * 64 * 4;
constexpr int kBandRows = 32;       // integral-image band height
constexpr int kBandRowsSmall = 16;  // ... for batches of <= kSmallBatch frames (one 1080p frame: 16 -> 0.1281-0.1287 ms vs 8 -> 0.1298-0.1305, 4 -> 0.131)
constexpr int kSmallBatch = 8;
// band height for batches > kSmallBatch: kBandRows, or SURFHIP_II_BAND (8..64)
inline int big_band_rows()
{
    static const int v = [] {
        const char* e = getenv("SURFHIP_II_BAND");
        const int b = e ? atoi(e) : kBandRows;
        return (b >= 8 && b <= 64) ? b : kBandRows;
    }();
    return v;
}
// band height for batches <= kSmallBatch: kBandRowsSmall, or
// SURFHIP_II_BAND_SMALL (4..32; A/B)
inline int small_band_rows()
{
    static const int v = [] {
        const char* e = getenv("SURFHIP_II_BAND_SMALL");
        const int b = e ? atoi(e) : kBandRowsSmall;
        return (b >= 4 && b <= 32) ? b : kBandRowsSmall;
    }();
    return v;
}
// colsum entries (per column) the integral of a batch of up to max_batch frames needs
inline long long integral_bands(int H, int max_batch)
{
    const int bb = big_band_rows(), sb = small_band_rows();
    const long long big = (long long)max_batch * ((H + bb - 1) / bb);
    const long long small = (long long)(max_batch < kSmallBatch ? max_batch : kSmallBatch) * ((H + sb - 1) / sb);
    return big > small ? big : small;
}
constexpr int kScanRows = 16;       // NMS block rows per scan workgroup (4 per wave)
constexpr int kItemCap = 64 * (kScanRows / 4);   // 2x2x2 blocks (= survivor slots) per scan item
constexpr int kCubeCap = 8;         // survivors per scan item whose fit inputs the scan records
constexpr int kCubeF = 20;          // floats per record (fit_quad's 19 responses + pad)

// Per-octave geometry and Hessian/NMS parameters, exactly as the reference
// host code derives them (surf.cpp:240-292, surfd.cu:2844-2865, 3062-3076).
struct OctaveParams {
    int sw, sh, sp, osize;          // response grid (swhp) and plane size
    long long ooff;                 // float offset of plane 0 in a frame block
    int octave, delta, init_scale, nscale;
    int mask[kMaxScale], b1[kMaxScale], x2[kMaxScale], x3[kMaxScale], x4[kMaxScale];
    float norm[kMaxScale];
    int borders[kMaxScale];         // host borders[] (d_borders), index s
    int mb[(kMaxScale - 2) / 2];    // NMS start offsets (maximum_borders, one per level)
    int nms_gx, nms_gy;             // NMS launch extent in threads
    // planes 0 and 1 of an octave > 0 are the reference's halfImage copies of
    // the previous octave's planes max_scale - 3 / max_scale - 1
    // (surf.cpp:252-258), never materialised: read in place at (r, c) ->
    // hbase[t] + r * hrow[t] + c * hcol[t] (floats).  With 4 scales plane
    // max_scale - 3 = 1 is itself a copy, so the chain is followed back to a
    // computed plane (stride 4, 8, ..).
    long long hbase[2];
    int hrow[2], hcol[2];
};

// Frame-level parameters (SurfParam + integral geometry).
struct FrameParams {
    int W, H, ip, iH;               // integral: (W+1) x (H+1), pitch ip ints
    long long ii_stride;            // ints per frame
    long long resp_stride;          // floats per frame
    int max_scale, init_lobe, sampling, noct;
    float thresh, divisor;
    int upright, extend, wsz, mag, osz, nfeat;
    int doubled;                    // the integral is of the 2x frame: describe at (2x, 2y)
};

struct Tables {
    float lut1[83];
    float lut2[40];
    float bins[72];
};

// ---- launch helpers (defined in surfhip_kernels.hip) -------------------
hipError_t set_tables(const Tables& t);

hipError_t launch_integral(const uint8_t* frames, int pitch, long long fstride, int nframes,
                           const FrameParams& P, uint32_t* colsum, int32_t* ii, hipStream_t s);
// Block ranges of the fused all-octave launches and the Hessian kernel of
// each octave (computed once per detector; make_plan).
struct LaunchPlan {
    int hess_start[kMaxOct + 1];    // k_hessian blocks of octave o: [start[o], start[o+1])
    int hess_nbx[kMaxOct];          // blocks per row of samples
    int nms_start[kMaxOct + 1];     // NMS blocks of octave o (every level)
    int nms_nbx[kMaxOct], nms_nby[kMaxOct];
    int q0, q0_strips;              // octave 0 on k_hess_q0 (u8 vertical streaming), 64-sample strips
    int p0;                         // ... on k_hess_p0 instead (producer + per-scale waves): its interval B; 0: q0
    int q1, q1_strips;              // octave 1 on k_hess_q1 (when k_hess_w is off)
    int q01;                        // q0 and q1 in one launch (k_hess_q01)
    int hw_n;                       // octaves 1 .. hw_n on k_hess_w (u8, shared strip integral); 0: off
    int hw_nstrips, hw_nblk;        // its strips per frame and blocks of 4 integral rows
    int t0, t0_nbx, t0_nby;         // octave 0 of the gather plan on k_hessian_t0 (LDS tiles): its blocks
    // A u8 Hessian kernel also writes the integral image (its producers'
    // strip integral plus the row sums left of the strip, k_ii_rowseg): no
    // separate integral pass.  Set when octaves 0-3 are on the u8 kernels
    // (p0 + k_hess_w); k_hessian octaves (past 3) run after them on the same
    // stream.  1: k_hess_w writes it (480-column strips), 2: k_hess_p0
    // (128-column strips).
    int iiw;
    int rs_rows;                    // rows per rowseg slab (4 x hw_nblk, zero past H)
    int rs_nstrips;                 // rowseg slabs per frame: the writer's strips
};
// the plan has kernels that read the u8 frames (not only the integral image)
inline bool plan_reads_frames(const LaunchPlan& p) { return p.q0 || p.q1 || p.hw_n > 0; }
// max_batch <= kGatherBatch (or SURFHIP_HESS_GATHER=1; =0 disables) puts every
// octave on the one-thread-per-response gather kernel: the streaming kernels
// walk whole strips, one wave each, too few waves to fill the chip for a few
// frames (measured crossover, 1080p: gather 9,956 vs streaming 7,981 frames/s
// at 8 frames, 12,474 vs 14,085 at 16).
constexpr int kGatherBatch = 8;
// float4s per k_worklist entry (k_describe_u2's flattened schedule)
constexpr int kWorkF4 = 3;
void make_plan(const FrameParams& P, const OctaveParams* oct, LaunchPlan& plan, int max_batch);
// the Hessian stage's kernels of a plan, as text (surfhip_hessian_plan)
std::string hessian_plan_text(const LaunchPlan& plan, const FrameParams& P);

// parts: 1 = the u8-frame kernels (frames must be given), 2 = the
// integral-image kernel (k_hessian), 3 = both; 4 / 8 = only the octave-0 /
// only the k_hess_w launch of part 1.  ii_out + rowseg (plan.iiw):
// k_hess_w (iiw 1) or k_hess_p0 (iiw 2) writes the frames' integral image
// into ii_out (rowseg: the k_ii_rowseg sums of the same frames); nullptr:
// neither does.
hipError_t launch_hessian(const uint8_t* frames, int pitch, long long fstride, const int32_t* ii, float* resp,
                          int nframes, const FrameParams& P, const OctaveParams* d_oct, const OctaveParams* h_oct,
                          const LaunchPlan& plan, hipStream_t s, int parts = 3, const uint32_t* rowseg = nullptr,
                          int32_t* ii_out = nullptr);
// plan.iiw: the row sums the writer's strips add to their integral (rowseg:
// nframes x rs_nstrips x rs_rows uint32; slab 0 and rows >= H stay zero)
hipError_t launch_rowseg(const uint8_t* frames, int pitch, long long fstride, int nframes, const FrameParams& P,
                         const LaunchPlan& plan, uint32_t* rowseg, hipStream_t s);
// NMS scan items: one wave's 64 block columns x kScanRows / 4 block rows;
// each item owns kItemCap survivor slots (no atomics in the scan).
// (also zeroes cand_count[0, nframes) and *status, the per-batch counters)
hipError_t launch_nms(const int32_t* ii, const float* resp, int nframes, const FrameParams& P,
                      const OctaveParams* d_oct, const LaunchPlan& plan, uint32_t* scan_key, uint32_t* scan_src,
                      float* scan_cube, int* item_count, int* item_off, surfhip_point* cand, uint32_t* keys,
                      int* cand_count, int cap, int* status, hipStream_t s, bool stash_trace);
hipError_t launch_sort(const surfhip_point* cand, const uint32_t* keys, uint64_t* gscratch,
                       const int* cand_count, const int* soff, int items_per_frame, int cap, int nframes,
                       surfhip_point* out, int max_pts, int* out_count, int* offsets, int* order, int* status,
                       hipStream_t s);
hipError_t set_max_lds(const void* fn, int bytes);
// queue: kDescQueueBytes of device scratch (the per-XCD work counters of
// k_describe_ur, 8 x kDescQ of them 256 B apart, zeroed by the launch)
// beside: another stream's kernels (the next batch's integral) run beside
// it, so the persistent grid leaves each CU a workgroup slot
// work: max_batch * max_pts * kWorkF4 float4 of scratch (k_describe_u2's flattened schedule)
// cus: compute units of the detector's device (sizes the persistent grid)
// trace: the fit left getTrace to the describe (trace_in_describe, the same
// call's stash_trace of launch_nms)
hipError_t launch_describe(const int32_t* ii, const FrameParams& P, surfhip_point* pts, int max_pts,
                           const int* counts, const int* offsets, const int* order, float4* work, int nframes,
                           float* desc, int* queue, hipStream_t s, bool beside, int cus, bool trace);
// Whether a batch of nframes describes on k_describe_u2 (upright 4 x 4
// windows, batches > kGatherBatch or SURFHIP_DESC_UR=0, packed worklist
// fields large enough), and whether its laplace sign (getTrace,
// surfd.cu:369-377) is then taken there, from the integral rows the
// keypoint's window brings into L2, instead of in k_nms_fit
// (SURFHIP_TRACE_DESC=0: in the fit, A/B)
bool describe_on_u2(const FrameParams& P, int nframes);
bool trace_in_describe(const FrameParams& P, int nframes);
// Doubled-image input (surfhip_double.hip): frames (W x H) -> D ((2W-2) x
// (2H-2) u8, row pitch dpitch, a multiple of 4).
// HBM stream-rate kernels (surfhip_stream.hip): mode 0 copy, 1 read, 2 write
hipError_t launch_stream(int mode, const void* src, void* dst, size_t bytes, int ncu, hipStream_t s);
hipError_t launch_double(const uint8_t* frames, int pitch, long long fstride, int nframes, int W, int H,
                         uint8_t* dst, int dpitch, long long dstride, hipStream_t s);
// Descriptor matching (surfhip_match.hip): scratch = match_scratch_bytes().
size_t match_scratch_bytes(int n1, int n2, int flags);
hipError_t launch_match(surfhip_point* pts1, const surfhip_point* pts2, const float* f1, const float* f2, int n1,
                        int n2, int nf, int flags, void* scratch, hipStream_t s);
hipError_t launch_pack(const surfhip_point* pts, const float* desc, const int* counts, const int* offsets,
                       int nframes, int max_pts, int nfeat, const int* status, size_t cap_bytes, uint8_t* slab,
                       hipStream_t s);

}  // namespace surfhip
