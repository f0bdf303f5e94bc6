// Micro-benchmark: per-wave and per-SIMD issue rate of v_add_f32, v_pk_add_f32,
// v_pk_fma_f32, v_add_u32 and ds_read_b64 on gfx950 (1, 2, 4 waves per SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2f __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ __launch_bounds__(256) void k(float* out, int iters)
{
    v2f a[8];
    float b[8];
    unsigned u[8];
    for (int i = 0; i < 8; i++) { a[i] = {threadIdx.x * 1.f + i, i * 2.f}; b[i] = threadIdx.x + i; u[i] = threadIdx.x * 7 + i; }
    const v2f c = {1.0001f, 0.9999f};
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (KIND == 0) asm volatile("v_add_f32 %0, %0, %0" : "+v"(b[i]));
            if (KIND == 1) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
            if (KIND == 2) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(c));
            if (KIND == 3) asm volatile("v_add_u32 %0, %0, %0" : "+v"(u[i]));
            if (KIND == 4) asm volatile("v_fma_f32 %0, %0, %0, %0" : "+v"(b[i]));
            if (KIND == 5) asm volatile("v_dot4_u32_u8 %0, %0, %0, %0" : "+v"(u[i]));
            if (KIND == 6) asm volatile("v_lshl_add_u32 %0, %0, 1, %0" : "+v"(u[i]));
            if (KIND == 7) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(b[i]));
            if (KIND == 8) asm volatile("s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(u[i]));
            if (KIND == 9) asm volatile("v_add3_u32 %0, %0, %0, %0" : "+v"(u[i]));
            if (KIND == 10) asm volatile("v_sub_f32 %0, %0, %0" : "+v"(b[i]));
        }
    }
    float s = 0;
    for (int i = 0; i < 8; i++) s += a[i].x + a[i].y + b[i] + (float)u[i];
    if (s == 123.f) out[threadIdx.x] = s;
}

int main()
{
    float* out;
    hipMalloc(&out, 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[] = {"v_add_f32", "v_pk_add_f32", "v_pk_fma_f32", "v_add_u32", "v_fma_f32", "v_dot4_u32_u8",
                           "v_lshl_add_u32", "v_cvt_f32_u32", "nop1+v_add_dpp", "v_add3_u32", "v_sub_f32"};
    const int iters = 20000;
    for (int kind = 0; kind < 11; kind++) {
        for (int wps : {1, 2, 4}) {
            // 256 CUs x 4 SIMDs x wps waves, 4 waves per workgroup
            const int blocks = 256 * wps;
            auto launch = [&]() {
                switch (kind) {
                    case 0: k<0><<<blocks, 256>>>(out, iters); break;
                    case 1: k<1><<<blocks, 256>>>(out, iters); break;
                    case 2: k<2><<<blocks, 256>>>(out, iters); break;
                    case 3: k<3><<<blocks, 256>>>(out, iters); break;
                    case 4: k<4><<<blocks, 256>>>(out, iters); break;
                    case 5: k<5><<<blocks, 256>>>(out, iters); break;
                    case 6: k<6><<<blocks, 256>>>(out, iters); break;
                    case 7: k<7><<<blocks, 256>>>(out, iters); break;
                    case 8: k<8><<<blocks, 256>>>(out, iters); break;
                    case 9: k<9><<<blocks, 256>>>(out, iters); break;
                    case 10: k<10><<<blocks, 256>>>(out, iters); break;
                }
            };
            launch();
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double instr_per_wave = (double)iters * 32;
            const double cyc = ms * 1e-3 * 2.4e9;
            printf("%-14s waves/SIMD %d: %.2f cycles per instr per wave, %.2f cycles per instr per SIMD\n", names[kind],
                   wps, cyc / instr_per_wave, cyc / (instr_per_wave * wps));
        }
    }
    return 0;
}
