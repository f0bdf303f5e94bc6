// buf_range.hip -- which part of a raw buffer access's offset the gfx950
// range check sees (the k_hess_p0 integral writer with
// the row offset in the scalar offset corrupted 256-frame batches).
//
// One 4.5-GiB allocation, zeroed; a raw buffer resource over NR bytes at
// BASE inside it.  Each case stores one marker dword per lane with a
// (voffset, soffset) pair, then a scan kernel lists every nonzero dword of
// the whole allocation (offsets relative to BASE).  Every address any case
// can form (BASE + soffset + voffset < 4.2 GiB) lies inside the allocation.
// Loads: the same pairs read a pattern and report what came back.
//
//   hipcc --offload-arch=gfx950 -O2 -o buf_range buf_range.hip && ./buf_range
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

typedef __amdgpu_buffer_rsrc_t rsrc_t;

__global__ void k_store(uint8_t* base, int nr, const uint32_t* vo, uint32_t so, uint32_t marker)
{
    const rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, nr, 0x00020000);
    const int l = threadIdx.x;
    __builtin_amdgcn_raw_buffer_store_b32(marker + (uint32_t)l, r, vo[l], so, 0);
}

__global__ void k_store16(uint8_t* base, int nr, const uint32_t* vo, uint32_t so, uint32_t marker)
{
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    const rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, nr, 0x00020000);
    const int l = threadIdx.x;
    const uint32_t m = marker + 4u * (uint32_t)l;
    __builtin_amdgcn_raw_buffer_store_b128(v4{m, m + 1, m + 2, m + 3}, r, vo[l], so, 0);
}

__global__ void k_load(const uint8_t* base, int nr, const uint32_t* vo, uint32_t so, uint32_t* out)
{
    const rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, nr, 0x00020000);
    const int l = threadIdx.x;
    out[l] = __builtin_amdgcn_raw_buffer_load_b32(r, vo[l], so, 0);
}

// every nonzero dword of [p, p + n): (index, value) appended, up to cap
__global__ void k_scan(const uint32_t* p, size_t n, unsigned long long* idx, uint32_t* val, uint32_t* cnt, uint32_t cap)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t v = p[i];
        if (v) {
            const uint32_t k = atomicAdd(cnt, 1u);
            if (k < cap) {
                idx[k] = i;
                val[k] = v;
            }
        }
    }
}

int main()
{
    const size_t TOTAL = 4608ull << 20;            // 4.5 GiB
    const size_t BASE = 64ull << 20;
    const int NR = 1 << 20;                        // 1 MiB resource
    uint8_t* buf;
    CK(hipMalloc(&buf, TOTAL));
    CK(hipMemset(buf, 0, TOTAL));
    uint32_t *dvo, *dout, *dval, *dcnt;
    unsigned long long* didx;
    const uint32_t CAP = 4096;
    CK(hipMalloc(&dvo, 64 * 4));
    CK(hipMalloc(&dout, 64 * 4));
    CK(hipMalloc(&didx, CAP * 8));
    CK(hipMalloc(&dval, CAP * 4));
    CK(hipMalloc(&dcnt, 4));

    struct Case {
        const char* name;
        uint32_t vbase, vstep, so;
        bool wide;
    };
    const uint32_t G = 0x40000000u;
    const Case cases[] = {
        {"A control: v = 4l, s = 0", 0, 4, 0, false},
        {"B v = 4l, s = NR - 128 (lanes >= 32: v + s >= NR)", 0, 4, (uint32_t)NR - 128, false},
        {"C v = 4l, s = NR", 0, 4, (uint32_t)NR, false},
        {"D v = 4l, s = NR + 8192 (k_hess_w's rows past H)", 0, 4, (uint32_t)NR + 8192, false},
        {"E v = 4l, s = 0x40000000 (k_hess_p0 SOFF rows above the frame)", 0, 4, G, false},
        {"F v = 0x40000000 + 4l, s = 0 (voffset past NR)", G, 4, 0, false},
        {"G v = 0x40000000 + 4l, s = 0x40000000 (sum 2^31)", G, 4, G, false},
        {"H v = 4l, s = 0x7fffff00", 0, 4, 0x7fffff00u, false},
        {"I v = 4l, s = 0x80000000", 0, 4, 0x80000000u, false},
        {"J v = 4l, s = 0xffffff80 (v + s wraps 2^32 for lanes >= 32)", 0, 4, 0xffffff80u, false},
        {"K v = NR - 8 + 4l, s = 0 (straddle, dword)", (uint32_t)NR - 8, 4, 0, false},
        {"L b128: v = NR - 24 + 16l, s = 0 (straddle, 16 B)", (uint32_t)NR - 24, 16, 0, true},
        {"M b128: v = 16l, s = NR - 24", 0, 16, (uint32_t)NR - 24, true},
        {"N b128: v = 16l, s = 0x40000000", 0, 16, G, true},
    };
    std::vector<uint32_t> hvo(64);
    int ci = 0;
    for (const Case& c : cases) {
        ci++;
        for (int l = 0; l < 64; l++) hvo[l] = c.vbase + c.vstep * (uint32_t)l;
        CK(hipMemcpy(dvo, hvo.data(), 256, hipMemcpyHostToDevice));
        const uint32_t marker = (uint32_t)ci << 24;
        if (c.wide)
            k_store16<<<1, 64>>>(buf + BASE, NR, dvo, c.so, marker);
        else
            k_store<<<1, 64>>>(buf + BASE, NR, dvo, c.so, marker);
        CK(hipDeviceSynchronize());
        CK(hipMemset(dcnt, 0, 4));
        k_scan<<<4096, 256>>>((const uint32_t*)buf, TOTAL / 4, didx, dval, dcnt, CAP);
        CK(hipDeviceSynchronize());
        uint32_t cnt;
        CK(hipMemcpy(&cnt, dcnt, 4, hipMemcpyDeviceToHost));
        const uint32_t n = cnt < CAP ? cnt : CAP;
        std::vector<unsigned long long> idx(n);
        std::vector<uint32_t> val(n);
        if (n) {
            CK(hipMemcpy(idx.data(), didx, n * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(val.data(), dval, n * 4, hipMemcpyDeviceToHost));
        }
        // lanes whose dword(s) landed, and where (offset from BASE)
        printf("%s\n  %u dwords landed", c.name, cnt);
        long long lo = 0, hi = 0;
        int lmin = 999, lmax = -1;
        for (uint32_t k = 0; k < n; k++) {
            const long long off = (long long)(idx[k] * 4) - (long long)BASE;
            const int lane = c.wide ? (int)((val[k] & 0xffffff) / 4) : (int)(val[k] & 0xffffff);
            if (k == 0 || off < lo) lo = off;
            if (k == 0 || off > hi) hi = off;
            if (lane < lmin) lmin = lane;
            if (lane > lmax) lmax = lane;
        }
        if (n) printf(": lanes %d..%d, offsets from base 0x%llx..0x%llx", lmin, lmax, lo, hi);
        printf("\n");
        for (uint32_t k = 0; k < n && k < 4; k++)
            printf("    lane %u at base%+lld\n", c.wide ? (val[k] & 0xffffff) / 4 : val[k] & 0xffffff,
                   (long long)(idx[k] * 4) - (long long)BASE);
        CK(hipMemset(buf, 0, TOTAL));
    }
    // loads: pattern p(o) = o | 1 for every dword in [BASE - 64 KiB, BASE + 2 NR)
    {
        std::vector<uint32_t> pat((2 * NR + 65536) / 4);
        for (size_t i = 0; i < pat.size(); i++) pat[i] = (uint32_t)(i * 4) | 1u;
        CK(hipMemcpy(buf + BASE - 65536, pat.data(), pat.size() * 4, hipMemcpyHostToDevice));
        const struct {
            const char* name;
            uint32_t vbase, so;
        } lc[] = {{"load v = 4l, s = 0", 0, 0},
                  {"load v = 4l, s = NR - 128", 0, (uint32_t)NR - 128},
                  {"load v = 4l, s = NR", 0, (uint32_t)NR},
                  {"load v = 4l, s = 0x40000000", 0, G},
                  {"load v = NR - 128 + 4l, s = 0", (uint32_t)NR - 128, 0},
                  {"load v = 4l - 65536 (wraps), s = 0", (uint32_t)-65536, 0}};
        for (auto& L : lc) {
            for (int l = 0; l < 64; l++) hvo[l] = L.vbase + 4u * (uint32_t)l;
            CK(hipMemcpy(dvo, hvo.data(), 256, hipMemcpyHostToDevice));
            k_load<<<1, 64>>>(buf + BASE, NR, dvo, L.so, dout);
            CK(hipDeviceSynchronize());
            uint32_t o[64];
            CK(hipMemcpy(o, dout, 256, hipMemcpyDeviceToHost));
            int nz = 0;
            for (int l = 0; l < 64; l++) nz += o[l] != 0;
            printf("%s: %d of 64 lanes nonzero; lane0 %#x lane31 %#x lane32 %#x lane63 %#x\n", L.name, nz, o[0], o[31],
                   o[32], o[63]);
        }
    }
    CK(hipFree(buf));
    printf("done\n");
    return 0;
}
