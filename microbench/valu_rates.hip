// Microbenchmark: VALU issue rates on gfx950 at 16 waves/CU (4 per SIMD).
// Each lane runs N iterations of 8 independent chains of one instruction kind.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 4096

template <int KIND>
__global__ __launch_bounds__(1024) void k(float* out, float a, float b) {
    __shared__ unsigned sh[16384];  // 64 KiB for the ds_read mix
    if (KIND == 40 && a < -1e30f) sh[threadIdx.x] = 1u;
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    unsigned u[8];
    for (int i = 0; i < 8; ++i) u[i] = threadIdx.x * 7919u + i;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (KIND == 0) {
                asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[i]) : "v"(a), "v"(b));
            }
            if constexpr (KIND == 1) {
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(*reinterpret_cast<double*>(&x[i & ~1])) : "v"(*(double*)&x[0]), "v"(*(double*)&x[2]));
            }
            if constexpr (KIND == 2) {
                asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "v"(u[(i + 3) & 7]));
            }
            if constexpr (KIND == 3) {
                asm volatile("v_sad_u16 %0, %1, %2, %0" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "v"(u[(i + 3) & 7]));
            }
            if constexpr (KIND == 4) {
                asm volatile("v_sad_u32 %0, %1, %2, %0" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "v"(u[(i + 3) & 7]));
            }
            if constexpr (KIND == 5) {
                asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
            }
            if constexpr (KIND == 6) {
                asm volatile("v_lshlrev_b32 %0, 7, %0" : "+v"(u[i]));
            }
            if constexpr (KIND == 7) {
                asm volatile("v_or_b32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
            }
            if constexpr (KIND == 8) {
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
            }
            if constexpr (KIND == 9) {
                asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "v"(u[(i + 2) & 7]));
            }
            if constexpr (KIND == 10) {
                asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
            }
            if constexpr (KIND == 11) {
                asm volatile("v_cvt_f32_ubyte1 %0, %1" : "=v"(x[i]) : "v"(u[i]));
            }
            if constexpr (KIND == 12) {
                asm volatile("v_cvt_f32_u32 %0, %1" : "=v"(x[i]) : "v"(u[i]));
            }
            if constexpr (KIND == 13) {
                asm volatile("v_mul_f32 %0, %1, %0" : "+v"(x[i]) : "v"(a));
            }
            if constexpr (KIND == 14) {
                asm volatile("v_add_f32 %0, %1, %0" : "+v"(x[i]) : "v"(a));
            }
            if constexpr (KIND == 15) {
                asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(*reinterpret_cast<double*>(&x[i & ~1])) : "v"(*(double*)&x[2]));
            }
            if constexpr (KIND == 16) {
                asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(*reinterpret_cast<double*>(&x[i & ~1])) : "v"(*(double*)&x[2]));
            }
            if constexpr (KIND == 17) {
                asm volatile("v_max_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
            }
            if constexpr (KIND == 18) {
                asm volatile("v_and_b32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
            }
            if constexpr (KIND == 19) {
                asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(u[i]));
            }
            if constexpr (KIND == 20) {
                asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "v"(u[(i + 2) & 7]));
            }
            if constexpr (KIND == 21) {
                asm volatile("v_dot4_u32_u8 %0, %1, %2, %0" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "v"(u[(i + 3) & 7]));
            }
            if constexpr (KIND == 22) {
                asm volatile("v_mov_b32 %0, %1" : "=v"(u[i]) : "v"(u[(i + 1) & 7]));
            }
            if constexpr (KIND == 23) {
                asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
            }
            if constexpr (KIND == 24) {
                asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[i]) : "v"(x[(i + 1) & 7]));
            }
            if constexpr (KIND == 25) {
                asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[i]) : "v"(x[(i + 1) & 7]));
            }
            if constexpr (KIND == 26) {
                asm volatile("v_add_f32_e64 %0, |%0|, |%1|" : "+v"(x[i]) : "v"(x[(i + 1) & 7]));
            }
            if constexpr (KIND == 27) {
                asm volatile("v_cvt_u32_f32 %0, %1" : "=v"(u[i]) : "v"(x[i]));
            }
            if constexpr (KIND == 28) {
                asm volatile("v_lshl_add_u32 %0, %0, 6, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
            }
            if constexpr (KIND == 29) {
                asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
            }
            if constexpr (KIND == 30) {
                asm volatile("v_pk_add_f32 %0, %0, %1 neg_lo:[0,1] neg_hi:[0,1]" : "+v"(*reinterpret_cast<double*>(&x[i & ~1])) : "v"(*(double*)&x[2]));
            }
            if constexpr (KIND == 31) {  // sad + fma alternating (slow + fast)
                if (i & 1) asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "v"(u[(i + 3) & 7]));
                else asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[i]) : "v"(a), "v"(b));
            }
            if constexpr (KIND == 32) {  // lshl_or + mul alternating
                if (i & 1) asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
                else asm volatile("v_mul_f32 %0, %1, %0" : "+v"(x[i]) : "v"(a));
            }
            if constexpr (KIND == 33) {  // bilateral pair: sad, lshl_or, mul, 3 fma, add + 1 fma (8 instrs)
                switch (i) {
                    case 0: asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(u[0]) : "v"(u[1]), "v"(u[3])); break;
                    case 1: asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(u[2]) : "v"(u[5])); break;
                    case 2: asm volatile("v_mul_f32 %0, %1, %0" : "+v"(x[0]) : "v"(a)); break;
                    case 3: asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[1]) : "v"(a), "v"(b)); break;
                    case 4: asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[2]) : "v"(a), "v"(b)); break;
                    case 5: asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[3]) : "v"(a), "v"(b)); break;
                    case 6: asm volatile("v_add_f32 %0, %1, %0" : "+v"(x[4]) : "v"(a)); break;
                    default: asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[5]) : "v"(a), "v"(b)); break;
                }
            }
            if constexpr (KIND == 34) {  // two slow ops alternating: cvt_f32_ubyte + sad
                if (i & 1) asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "v"(u[(i + 3) & 7]));
                else asm volatile("v_cvt_f32_ubyte1 %0, %1" : "=v"(x[i]) : "v"(u[i]));
            }
            if constexpr (KIND == 36) {  // pk_fma / sad 1:1
                if (i & 1) asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "v"(u[(i + 3) & 7]));
                else asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(*reinterpret_cast<double*>(&x[i & ~1])) : "v"(*(double*)&x[0]), "v"(*(double*)&x[2]));
            }
            if constexpr (KIND == 37) {  // pk_fma / fma 1:1
                if (i & 1) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[i]) : "v"(a), "v"(b));
                else asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(*reinterpret_cast<double*>(&x[i & ~1])) : "v"(*(double*)&x[0]), "v"(*(double*)&x[2]));
            }
            if constexpr (KIND == 38) {  // sad, lshl_or, pk_fma, pk_fma x2
                switch (i & 3) {
                    case 0: asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "v"(u[(i + 3) & 7])); break;
                    case 1: asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7])); break;
                    default: asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(*reinterpret_cast<double*>(&x[(i & 1) * 2 + 4])) : "v"(*(double*)&x[0]), "v"(*(double*)&x[2])); break;
                }
            }
            if constexpr (KIND == 39) {  // pk_mul / mul 1:1 and pk_add
                if (i & 1) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(x[i]) : "v"(a));
                else asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(*reinterpret_cast<double*>(&x[i & ~1])) : "v"(*(double*)&x[2]));
            }
            if constexpr (KIND == 40) {  // ds_read_b32 + fma 1:3 (LDS issue alongside VALU)
                if ((i & 3) == 0) { asm volatile("ds_read_b32 %0, %1" : "=v"(u[i]) : "v"(u[(i+1)&7] & 0xfffcu)); }
                else asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[i]) : "v"(a), "v"(b));
                if (i == 7) asm volatile("s_waitcnt lgkmcnt(0)");
            }
            if constexpr (KIND == 41) {  // f16 (lo half) x f32 + f32 -> f32
                asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(x[i]) : "v"(u[(i + 1) & 7]), "v"(a));
            }
            if constexpr (KIND == 42) {  // folded JBF tap on an f16 source plane: sad, min, lshl_or,
                                         // 3 fma_mix, add (+ 1 fma_mix to make 8)
                switch (i) {
                    case 0: asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(u[0]) : "v"(u[1]), "v"(u[3])); break;
                    case 1: asm volatile("v_min_u32 %0, %0, %1" : "+v"(u[2]) : "v"(u[5])); break;
                    case 2: asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(u[4]) : "v"(u[5])); break;
                    case 3: asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(x[1]) : "v"(u[6]), "v"(a)); break;
                    case 4: asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(x[2]) : "v"(u[6]), "v"(a)); break;
                    case 5: asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(x[3]) : "v"(u[7]), "v"(a)); break;
                    case 6: asm volatile("v_add_f32 %0, %1, %0" : "+v"(x[4]) : "v"(a)); break;
                    default: asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(x[5]) : "v"(u[6]), "v"(a)); break;
                }
            }
            if constexpr (KIND == 43) {  // fma_mix / fma 1:1
                if (i & 1) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[i]) : "v"(a), "v"(b));
                else asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(x[i]) : "v"(u[(i + 1) & 7]), "v"(a));
            }
            if constexpr (KIND == 44) {  // fma_mix / sad 1:1
                if (i & 1) asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "v"(u[(i + 3) & 7]));
                else asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(x[i]) : "v"(u[(i + 1) & 7]), "v"(a));
            }
            if constexpr (KIND == 35) {  // 1 slow : 3 fast
                if ((i & 3) == 0) asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "v"(u[(i + 3) & 7]));
                else asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[i]) : "v"(a), "v"(b));
            }
        }
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i] + (float)u[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND>
double run(const char* name, float* d, int blocks, int pk) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(1024), 0, 0, d, 1.0001f, 0.5f);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(1024), 0, 0, d, 1.0001f, 0.5f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double insts = 5.0 * blocks * 16.0 /*waves*/ * ITERS * 8;  // wave-instructions
    double per_simd_cycles_ns = ms * 1e6 / (insts / (256.0 * 4));  // ns per wave-instr per SIMD
    printf("%-22s %8.3f ms  %.3f ns per wave-instr per SIMD (= %.2f cycles at 2.4 GHz)%s\n", name, ms / 5, per_simd_cycles_ns,
           per_simd_cycles_ns * 2.4, pk ? "  [2 f32 per lane]" : "");
    return ms;
}

int main() {
    float* d; hipMalloc(&d, 256 * 1024 * 4 * sizeof(float));
    int blocks = 256;  // one 1024-thread block per CU
    run<0>("v_fma_f32", d, blocks, 0);
    run<1>("v_pk_fma_f32", d, blocks, 1);
    run<2>("v_sad_u8", d, blocks, 0);
    run<3>("v_sad_u16", d, blocks, 0);
    run<4>("v_sad_u32", d, blocks, 0);
    run<5>("v_lshl_or_b32", d, blocks, 0);
    run<6>("v_lshlrev_b32 (VOP2)", d, blocks, 0);
    run<7>("v_or_b32 (VOP2)", d, blocks, 0);
    run<8>("v_add_u32 (VOP2)", d, blocks, 0);
    run<9>("v_mad_u32_u24", d, blocks, 0);
    run<10>("v_mul_u32_u24 (VOP2)", d, blocks, 0);
    run<11>("v_cvt_f32_ubyte1", d, blocks, 0);
    run<12>("v_cvt_f32_u32", d, blocks, 0);
    run<13>("v_mul_f32", d, blocks, 0);
    run<14>("v_add_f32", d, blocks, 0);
    run<15>("v_pk_mul_f32", d, blocks, 1);
    run<16>("v_pk_add_f32", d, blocks, 1);
    run<17>("v_max_u32 (VOP2)", d, blocks, 0);
    run<18>("v_and_b32 (VOP2)", d, blocks, 0);
    run<19>("v_bfe_u32", d, blocks, 0);
    run<20>("v_perm_b32", d, blocks, 0);
    run<21>("v_dot4_u32_u8", d, blocks, 0);
    run<22>("v_mov_b32", d, blocks, 0);
    run<23>("v_cndmask_b32", d, blocks, 0);
    run<24>("v_max_f32", d, blocks, 0);
    run<25>("v_sub_f32", d, blocks, 0);
    run<26>("v_add_f32_e64 |a|+|b|", d, blocks, 0);
    run<27>("v_cvt_u32_f32", d, blocks, 0);
    run<28>("v_lshl_add_u32", d, blocks, 0);
    run<29>("v_fmac_f32 (VOP2)", d, blocks, 0);
    run<30>("v_pk_add_f32 neg", d, blocks, 1);
    run<31>("mix sad/fma 1:1", d, blocks, 0);
    run<32>("mix lshl_or/mul 1:1", d, blocks, 0);
    run<33>("mix bilateral pair 8", d, blocks, 0);
    run<34>("mix cvt/sad 1:1", d, blocks, 0);
    run<35>("mix sad/fma 1:3", d, blocks, 0);
    run<36>("mix pk_fma/sad 1:1", d, blocks, 0);
    run<37>("mix pk_fma/fma 1:1", d, blocks, 0);
    run<38>("mix sad,lshl_or,2 pk_fma", d, blocks, 0);
    run<39>("mix pk_mul/mul 1:1", d, blocks, 0);
    run<40>("mix ds_read/fma 1:3", d, blocks, 0);
    run<41>("v_fma_mix_f32", d, blocks, 0);
    run<42>("mix folded f16 JBF tap 8", d, blocks, 0);
    run<43>("mix fma_mix/fma 1:1", d, blocks, 0);
    run<44>("mix fma_mix/sad 1:1", d, blocks, 0);
    run<33>("mix bilateral pair 8", d, blocks, 0);
    return 0;
}
