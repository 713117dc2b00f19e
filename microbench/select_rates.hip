// Microbenchmark: select / compare / min-max issue rates on gfx950 at 16 waves per CU
// (4 per SIMD), 8 independent chains per lane (as valu_rates.hip). Question: is
// v_cndmask_b32 (valu_rates.hip: 9.3 ns per wave-instruction back to back) really that
// slow, and with which condition source; what do select-free forms cost instead.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 4096

template <int KIND>
__global__ __launch_bounds__(1024) void k(float* out, float a, float b) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    unsigned u[8];
    for (int i = 0; i < 8; ++i) u[i] = threadIdx.x * 7919u + i;
    unsigned long long m0 = 0x5555555555555555ull ^ (unsigned long long)blockIdx.x;  // an SGPR-pair mask
    asm volatile("" : "+s"(m0));
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (KIND == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[i]) : "v"(a), "v"(b));
            if constexpr (KIND == 1)  // condition in VCC, set once per 8 by a compare
            {
                if (i == 0) asm volatile("v_cmp_lt_u32 vcc, %0, %1" : : "v"(u[1]), "v"(u[2]) : "vcc");
                asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(u[(i + 1) & 7]) : "vcc");
            }
            if constexpr (KIND == 2)  // condition in an SGPR pair (VOP3 form)
                asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "s"(m0));
            if constexpr (KIND == 3) {  // compare + select pairs (the argmin pattern)
                asm volatile("v_cmp_eq_u32 vcc, %0, %1\n\tv_cndmask_b32 %2, %2, %3, vcc"
                             : : "v"(u[(i + 1) & 7]), "v"(u[(i + 2) & 7]), "v"(u[i]), "v"(u[(i + 3) & 7]) : "vcc");
            }
            if constexpr (KIND == 4) {  // compare to an SGPR pair + VOP3 select
                unsigned long long c;
                asm volatile("v_cmp_eq_u32_e64 %0, %1, %2" : "=s"(c) : "v"(u[(i + 1) & 7]), "v"(u[(i + 2) & 7]));
                asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[(i + 3) & 7]), "s"(c));
            }
            if constexpr (KIND == 5) asm volatile("v_min_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
            if constexpr (KIND == 6) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "v"(u[(i + 2) & 7]));
            if constexpr (KIND == 7) asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "v"(u[(i + 2) & 7]));
            if constexpr (KIND == 8) asm volatile("v_cmp_eq_u32 vcc, %0, %1" : : "v"(u[(i + 1) & 7]), "v"(u[i]) : "vcc");
            if constexpr (KIND == 9) {  // cndmask 1 : 3 fma
                if ((i & 3) == 0) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "s"(m0));
                else asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[i]) : "v"(a), "v"(b));
            }
            if constexpr (KIND == 10) {  // cmp+cndmask 1 : 2 fma
                if ((i & 3) == 0)
                    asm volatile("v_cmp_eq_u32 vcc, %0, %1\n\tv_cndmask_b32 %2, %2, %3, vcc"
                                 : : "v"(u[(i + 1) & 7]), "v"(u[(i + 2) & 7]), "v"(u[i]), "v"(u[(i + 3) & 7]) : "vcc");
                else if (i & 1) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[i]) : "v"(a), "v"(b));
            }
            if constexpr (KIND == 11) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
            if constexpr (KIND == 12) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "v"(u[(i + 2) & 7]));
            if constexpr (KIND == 13) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(*reinterpret_cast<double*>(&x[i & ~1])) : "v"(*(double*)&x[0]), "v"(*(double*)&x[2]));
            if constexpr (KIND == 14) asm volatile("v_sqrt_f32 %0, %1" : "=v"(x[i]) : "v"(x[(i + 1) & 7]));
            if constexpr (KIND == 15) asm volatile("v_rcp_f32 %0, %1" : "=v"(x[i]) : "v"(x[(i + 1) & 7]));
            if constexpr (KIND == 16) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(*reinterpret_cast<double*>(&x[i & ~1])) : "v"(x[(i + 1) & 7]));
            if constexpr (KIND == 17) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
        }
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i] + (float)u[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND>
void run(const char* name, float* d, int per8) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256;  // one 1024-thread workgroup per CU
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(1024), 0, 0, d, 1.0001f, 0.5f);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(1024), 0, 0, d, 1.0001f, 0.5f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double insts = 5.0 * blocks * 16.0 * ITERS * per8;  // wave-instructions
    const double ns = ms * 1e6 / (insts / (256.0 * 4));
    printf("%-34s %8.3f ms  %.3f ns per wave-instr per SIMD (%d instr per 8)\n", name, ms / 5, ns, per8);
}

int main() {
    float* d;
    hipMalloc(&d, 256 * 1024 * sizeof(float));
    run<0>("v_fma_f32", d, 8);
    run<1>("v_cndmask_b32 vcc (+1 v_cmp per 8)", d, 9);
    run<2>("v_cndmask_b32_e64 sgpr pair", d, 8);
    run<3>("v_cmp_eq_u32 vcc + v_cndmask pair", d, 16);
    run<4>("v_cmp_eq_u32_e64 sgpr + cndmask_e64", d, 16);
    run<5>("v_min_u32", d, 8);
    run<6>("v_min3_u32", d, 8);
    run<7>("v_med3_u32", d, 8);
    run<8>("v_cmp_eq_u32 vcc", d, 8);
    run<9>("mix cndmask_e64 1 : fma 3", d, 8);
    run<10>("mix cmp+cndmask 1 : fma 2", d, 6);
    run<11>("v_sub_u32", d, 8);
    run<12>("v_max3_u32", d, 8);
    run<13>("v_fma_f64", d, 8);
    run<14>("v_sqrt_f32", d, 8);
    run<15>("v_rcp_f32", d, 8);
    run<16>("v_cvt_f64_f32", d, 8);
    run<17>("v_pk_max_u16", d, 8);
    run<0>("v_fma_f32 (again)", d, 8);
    return 0;
}
