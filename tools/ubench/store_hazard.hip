// store_hazard.hip -- does a VALU write of a 16-B buffer store's data VGPRs,
// issued right after the store, change what the store writes, and does it
// matter whether the store's scalar offset is an SGPR or the constant 0?
// (k_hess_p0's integral stores with the row offset in an
// SGPR soffset left wrong values in 256-frame batches; the range check sees
// the soffset (buf_range.hip), so the stores were not misplaced.)
//
// LLVM's hazard recognizer requires one wait state between a store of more
// than 8 bytes and a VALU write of its data registers only when the store's
// soffset is NOT a register (GCNHazardRecognizer::createsVALUHazard); with
// an SGPR soffset it lets the compiler schedule the overwrite right after the
// store.  Here the sequence is fixed by inline asm:
//   v[40:43] = pattern; buffer_store_dwordx4 v[40:43]; [s_nop 0]; v[40:43] = -1
// over many waves and iterations; the host counts stored dwords that are not
// the pattern.
//
//   hipcc --offload-arch=gfx950 -O2 -o store_hazard store_hazard.hip && ./store_hazard
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

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int ITER = 64;

// FORM: 0 buffer_store_dwordx4, SGPR soffset; 1 buffer_store_dwordx4,
// constant-0 soffset (the offset in the VGPR); 2 global_store_dwordx4;
// 3 buffer_store_dwordx2 (constant soffset); 4 buffer_store_dwordx3.
// GAP: what sits between the store and the first overwrite: "" (nothing),
// s_nop N (N + 1 wait states) or independent VALU instructions.
#define HZ_BODY(STORE, GAP, ...)                                                                    \
    asm volatile("v_mov_b32 v40, %0\n\t"                                                           \
                 "v_add_u32 v41, 1, %0\n\t"                                                        \
                 "v_add_u32 v42, 2, %0\n\t"                                                        \
                 "v_add_u32 v43, 3, %0\n\t"                                                        \
                 "s_nop 4\n\t" STORE "\n\t" GAP                                                     \
                 "v_mov_b32 v40, -1\n\t"                                                           \
                 "v_mov_b32 v41, -1\n\t"                                                           \
                 "v_mov_b32 v42, -1\n\t"                                                           \
                 "v_mov_b32 v43, -1\n\t" ::"v"(m), __VA_ARGS__                                     \
                 : "v40", "v41", "v42", "v43", "v44", "v45", "memory")
#define HZ_KERNEL(NAME, STORE, GAP, ...)                                                            \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t nbytes)                     \
    {                                                                                               \
        const uint64_t p = (uint64_t)(uintptr_t)out;                                                \
        const v4i rs = {(int)(uint32_t)p, (int)(uint32_t)(p >> 32), (int)nbytes, 0x00020000};      \
        const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;                                   \
        const uint32_t nthr = gridDim.x * blockDim.x;                                               \
        for (int i = 0; i < ITER; i++) {                                                            \
            const uint32_t m = ((uint32_t)i * nthr + t) * 4u + 1u;                                  \
            const uint32_t row = (uint32_t)i * nthr * 16u, col = t * 16u;                           \
            uint32_t* gp = out + ((size_t)i * nthr + t) * 4;                                        \
            (void)rs; (void)row; (void)col; (void)gp;                                               \
            HZ_BODY(STORE, GAP, __VA_ARGS__);                                                       \
        }                                                                                           \
    }
#define SB4 "buffer_store_dwordx4 v[40:43], %1, %2, %3 offen"
#define CB4 "buffer_store_dwordx4 v[40:43], %1, %2, 0 offen"
#define GB4 "global_store_dwordx4 %1, v[40:43], off"
#define CB2 "buffer_store_dwordx2 v[40:41], %1, %2, 0 offen"
#define CB3 "buffer_store_dwordx3 v[40:42], %1, %2, 0 offen"
#define SARGS "v"(col), "s"(rs), "s"(row)
#define CARGS "v"(col + row), "s"(rs)
#define GARGS "v"(gp)
#define VALU1 "v_add_u32 v44, 1, v44\n\t"
HZ_KERNEL(k_s_0, SB4, "", SARGS)
HZ_KERNEL(k_s_n0, SB4, "s_nop 0\n\t", SARGS)
HZ_KERNEL(k_s_n1, SB4, "s_nop 1\n\t", SARGS)
HZ_KERNEL(k_c_0, CB4, "", CARGS)
HZ_KERNEL(k_c_n0, CB4, "s_nop 0\n\t", CARGS)
HZ_KERNEL(k_c_n1, CB4, "s_nop 1\n\t", CARGS)
HZ_KERNEL(k_c_n2, CB4, "s_nop 2\n\t", CARGS)
HZ_KERNEL(k_c_n4, CB4, "s_nop 4\n\t", CARGS)
HZ_KERNEL(k_c_v1, CB4, VALU1, CARGS)
HZ_KERNEL(k_c_v2, CB4, VALU1 VALU1, CARGS)
HZ_KERNEL(k_c_v4, CB4, VALU1 VALU1 VALU1 VALU1, CARGS)
HZ_KERNEL(k_g_0, GB4, "", GARGS)
HZ_KERNEL(k_g_n0, GB4, "s_nop 0\n\t", GARGS)
HZ_KERNEL(k_g_n1, GB4, "s_nop 1\n\t", GARGS)
HZ_KERNEL(k_c2_0, CB2, "", CARGS)
HZ_KERNEL(k_c3_0, CB3, "", CARGS)
HZ_KERNEL(k_c3_n0, CB3, "s_nop 0\n\t", CARGS)

int main()
{
    const int nb = 2048, nt = 256;
    const uint32_t nthr = (uint32_t)nb * nt;
    const size_t n = (size_t)nthr * ITER * 4;                 // dwords
    uint32_t* d;
    CK(hipMalloc(&d, n * 4));
    std::vector<uint32_t> h(n);
    struct K {
        void (*k)(uint32_t*, uint32_t);
        const char* name;
        int width;                                            // dwords stored per lane
    } ks[] = {{k_s_0, "buffer x4, SGPR soffset, overwrite next", 4},
              {k_s_n0, "buffer x4, SGPR soffset, s_nop 0 (1 wait state)", 4},
              {k_s_n1, "buffer x4, SGPR soffset, s_nop 1 (2)", 4},
              {k_c_0, "buffer x4, soffset 0, overwrite next", 4},
              {k_c_n0, "buffer x4, soffset 0, s_nop 0 (1)", 4},
              {k_c_n1, "buffer x4, soffset 0, s_nop 1 (2)", 4},
              {k_c_n2, "buffer x4, soffset 0, s_nop 2 (3)", 4},
              {k_c_n4, "buffer x4, soffset 0, s_nop 4 (5)", 4},
              {k_c_v1, "buffer x4, soffset 0, 1 independent VALU", 4},
              {k_c_v2, "buffer x4, soffset 0, 2 independent VALU", 4},
              {k_c_v4, "buffer x4, soffset 0, 4 independent VALU", 4},
              {k_g_0, "global x4, overwrite next", 4},
              {k_g_n0, "global x4, s_nop 0 (1)", 4},
              {k_g_n1, "global x4, s_nop 1 (2)", 4},
              {k_c2_0, "buffer x2, soffset 0, overwrite next", 2},
              {k_c3_0, "buffer x3, soffset 0, overwrite next", 3},
              {k_c3_n0, "buffer x3, soffset 0, s_nop 0 (1)", 3}};
    for (const K& k : ks) {
        long long bad = 0, neg = 0, tot = 0;
        for (int rep = 0; rep < 4; rep++) {
            CK(hipMemset(d, 0, n * 4));
            k.k<<<nb, nt>>>(d, (uint32_t)(n * 4));
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < n; i++) {
                if ((int)(i & 3) >= k.width) continue;
                tot++;
                const uint32_t want = (uint32_t)((i / 4) * 4 + 1 + (i & 3));
                if (h[i] != want) {
                    bad++;
                    neg += h[i] == 0xffffffffu;
                }
            }
        }
        printf("%-52s %10lld of %lld dwords wrong (%lld hold the overwrite)\n", k.name, bad, tot, neg);
        fflush(stdout);
    }
    CK(hipFree(d));
    return 0;
}
