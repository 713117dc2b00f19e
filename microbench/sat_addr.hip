// Microbenchmark + semantics check: a saturating 16-bit multiply-add as the colour-LUT
// address of the joint bilateral taps (gfx950).
//
// Question 1 (semantics): v_mad_u16 / v_mad_legacy_u16 with the clamp bit -- is the
// result min(d * S + B, 65535) for every d <= 1023 (the product computed wide before the
// clamp), and what happens to the high 16 bits of the destination VGPR (zeroed or kept)?
// Question 2 (issue rate): the folded JBF tap as sad + mad_u16(clamp) + 3 fma + add
// (6 VALU) against today's sad + lshl_or + mul + 3 fma + add (7 VALU) and the clamped
// fold sad + min + lshl_or + 3 fma + add (7 VALU), 16 waves per CU, 8 independent taps.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define ITERS 2048

template <int KIND>
__global__ __launch_bounds__(1024) void sem(unsigned* out, unsigned S, unsigned B) {
    const unsigned d = threadIdx.x;  // 0..1023
    const unsigned pre = 0xdead0000u | (d & 0xffffu);
    unsigned r;
    if constexpr (KIND == 0)
        asm volatile("v_mov_b32 %0, %1\n\ts_nop 1\n\tv_mad_u16 %0, %2, %3, %4 clamp" : "=&v"(r) : "v"(pre), "v"(d), "s"(S), "v"(B));
    else
        asm volatile("v_mov_b32 %0, %1\n\ts_nop 1\n\tv_mad_legacy_u16 %0, %2, %3, %4 clamp" : "=&v"(r) : "v"(pre), "v"(d), "s"(S), "v"(B));
    out[d] = r;
}

template <int KIND>
__global__ __launch_bounds__(1024) void rate(float* out, float a, unsigned S) {
    float s0[8], s1[8], s2[8], sk[8];
    unsigned c[8], g[8];
    for (int i = 0; i < 8; ++i) {
        s0[i] = s1[i] = s2[i] = sk[i] = threadIdx.x * 0.001f + i;
        c[i] = threadIdx.x * 0x01030507u + i;
        g[i] = threadIdx.x * 0x07050301u + 3 * i;
    }
    const unsigned lane4 = (threadIdx.x & 31) << 2;
    const float p0 = 1.f, p1 = 2.f, p2 = 3.f;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            unsigned d, ad;
            float w;
            asm volatile("v_sad_u8 %0, %1, %2, 0" : "=v"(d) : "v"(g[i]), "v"(c[i]));
            if constexpr (KIND == 0) {  // today: lshl_or + mul (the LUT read is replaced by a cvt-free stand-in)
                asm volatile("v_lshl_or_b32 %0, %1, 7, %2" : "=v"(ad) : "v"(d), "v"(lane4));
                asm volatile("v_mul_f32 %0, %1, %2" : "=v"(w) : "v"(__uint_as_float(ad)), "s"(a));
            } else if constexpr (KIND == 1) {  // clamped fold: min + lshl_or
                asm volatile("v_min_u32 %0, 31, %1" : "=v"(ad) : "v"(d));
                asm volatile("v_lshl_or_b32 %0, %1, 7, %2" : "=v"(ad) : "v"(ad), "v"(lane4));
                w = __uint_as_float(ad);
            } else if constexpr (KIND == 2) {  // saturating fold: one mad_u16
                asm volatile("v_mad_u16 %0, %1, %2, %3 clamp" : "=v"(ad) : "v"(d), "s"(S), "v"(lane4));
                w = __uint_as_float(ad);
            } else {
                asm volatile("v_mad_legacy_u16 %0, %1, %2, %3 clamp" : "=v"(ad) : "v"(d), "s"(S), "v"(lane4));
                w = __uint_as_float(ad);
            }
            asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(s0[i]) : "v"(p0), "v"(w));
            asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(s1[i]) : "v"(p1), "v"(w));
            asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(s2[i]) : "v"(p2), "v"(w));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(sk[i]) : "v"(w));
        }
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += s0[i] + s1[i] + s2[i] + sk[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND>
void run_rate(const char* name, float* d, int per_tap) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256;
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(rate<KIND>, dim3(blocks), dim3(1024), 0, 0, d, 1.0001f, 1280u);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(rate<KIND>, dim3(blocks), dim3(1024), 0, 0, d, 1.0001f, 1280u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double taps = 5.0 * blocks * 16.0 * ITERS * 8;  // wave-taps
    const double ns_tap = ms * 1e6 / (taps / (256.0 * 4));
    printf("%-44s %8.3f ms  %.3f ns per wave-tap per SIMD, %.3f ns per instruction (%d per tap)\n", name, ms / 5,
           ns_tap, ns_tap / per_tap, per_tap);
}

template <int KIND>
int check_sem(const char* name, unsigned* d_out, unsigned S, unsigned B) {
    hipLaunchKernelGGL(sem<KIND>, dim3(1), dim3(1024), 0, 0, d_out, S, B);
    unsigned h[1024];
    if (hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int bad = 0, hi_kept = 0, hi_zero = 0;
    for (unsigned d = 0; d < 1024; ++d) {
        const unsigned long long want = (unsigned long long)d * S + B;
        const unsigned lo = want > 65535 ? 65535u : (unsigned)want;
        if ((h[d] & 0xffffu) != lo) {
            if (bad < 4) printf("  %s d=%u: got 0x%08x want lo 0x%04x\n", name, d, h[d], lo);
            ++bad;
        }
        hi_kept += (h[d] >> 16) == 0xdeadu;
        hi_zero += (h[d] >> 16) == 0;
    }
    printf("%-20s S=%u B=%u: low16 mismatches %d / 1024; high16 kept %d, zeroed %d\n", name, S, B, bad, hi_kept, hi_zero);
    return bad;
}

int main() {
    unsigned* d_out;
    float* d_f;
    hipMalloc(&d_out, 1024 * sizeof(unsigned));
    hipMalloc(&d_f, 256 * 1024 * sizeof(float));
    int bad = 0;
    bad += check_sem<0>("v_mad_u16 clamp", d_out, 1280, 33411);
    bad += check_sem<1>("v_mad_legacy_u16 clamp", d_out, 1280, 33411);
    bad += check_sem<0>("v_mad_u16 clamp", d_out, 2688, 131);
    bad += check_sem<1>("v_mad_legacy_u16 clamp", d_out, 2688, 131);
    run_rate<0>("sad lshl_or mul 3fma add (today, 7)", d_f, 7);
    run_rate<1>("sad min lshl_or 3fma add (clamped fold, 7)", d_f, 7);
    run_rate<2>("sad mad_u16 3fma add (saturating fold, 6)", d_f, 6);
    run_rate<3>("sad mad_legacy_u16 3fma add (6)", d_f, 6);
    run_rate<0>("today again", d_f, 7);
    printf("semantic mismatches: %d\n", bad);
    return 0;
}
