// Issue cost of the texture guide's exp: the shipped f64 evaluation
// (vip::exp_tab_f32: (float)exp((double)x) for every float x in [0, 32), 64-entry double
// table, 11 f64-class ops) against an f32 double-float evaluation that a correctly rounded
// result would need (2^(k/64) table as float pairs, Cody-Waite reduction to a float-float r,
// degree-4 polynomial, Ziv rounding test; the rare uncertain lanes would then take the f64
// path, not timed here), and the hardware v_exp_f32 (inexact; the lower bound).
// 16 waves per CU, 8 independent evaluations per lane per iteration; ns per evaluation per
// wave per SIMD. Timing only: the f32 form's values are not checked.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define HC(x)                                                               \
    do {                                                                    \
        const hipError_t e_ = (x);                                          \
        if (e_ != hipSuccess) {                                             \
            std::printf("%s -> %s\n", #x, hipGetErrorString(e_));          \
            std::exit(1);                                                   \
        }                                                                   \
    } while (0)

#include "vip_stencil.hpp"

#define ITERS 512

__device__ __forceinline__ float exp_ff_f32(float x, const float2* tab) {
    constexpr float kInvL = 0x1.715476p+6f;     // 64 / ln2
    constexpr float L1 = 0x1.62ep-7f;           // ln2 / 64, 12 significant bits (k * L1 exact)
    constexpr float L2 = 0x1.0bfbe8p-23f;       // next 24 bits
    constexpr float L3 = -0x1.1cf79ap-48f;      // the rest
    const float kf = __builtin_rintf(x * kInvL);
    const int k = (int)kf;
    const float r0 = __builtin_fmaf(-kf, L1, x);  // exact (Sterbenz)
    const float ph = kf * L2;
    const float pl = __builtin_fmaf(kf, L2, -ph);
    const float rh = r0 - ph;                     // two-sum of r0 and -ph
    const float bb = rh - r0;
    const float rl = ((r0 - (rh - bb)) + (-ph - bb)) - __builtin_fmaf(kf, L3, pl);
    // exp(r) - 1 = r + r^2 (1/2 + r/6 + r^2/24), the r term as the pair (rh, rl)
    float q = __builtin_fmaf(rh, 1.f / 24, 1.f / 6);
    q = __builtin_fmaf(rh, q, 0.5f);
    const float t = __builtin_fmaf(rh * rh, q, rl);
    const float2 T = tab[k & 63];                 // 2^(j/64) as (hi, lo)
    const float hi = __builtin_fmaf(T.x, rh, T.x);
    const float e1 = __builtin_fmaf(T.x, rh, T.x - hi);
    float lo = __builtin_fmaf(T.x, t, T.y);
    lo = __builtin_fmaf(T.y, rh, lo) + e1;
    // Ziv: the result is correctly rounded when hi + (lo -+ bound) round alike
    const float a = hi + (lo + hi * 0x1p-38f), b = hi + (lo - hi * 0x1p-38f);
    const float res = a == b ? a : __builtin_nanf("");
    return __builtin_ldexpf(res, k >> 6);
}

template <int KIND>
__global__ __launch_bounds__(1024) void rate(float* out, float seed) {
    __shared__ double etab[64];
    __shared__ float2 ftab[64];
    if (threadIdx.x < 64) {
        etab[threadIdx.x] = vip::kExp2Tab64[threadIdx.x];
        const double v = vip::kExp2Tab64[threadIdx.x];
        ftab[threadIdx.x] = make_float2((float)v, (float)(v - (double)(float)v));
    }
    __syncthreads();
    float x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = seed + 0.37f * i + 1e-5f * threadIdx.x;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float e;
            if constexpr (KIND == 0) e = vip::exp_tab_f32(x[i], etab);
            else if constexpr (KIND == 1) e = exp_ff_f32(x[i], ftab);
            else e = __builtin_amdgcn_exp2f(x[i] * 1.44269504f);
            x[i] = __builtin_fmaf(e, 0x1p-40f, x[i]);  // a dependence, x stays in [0, 32)
        }
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 1024 + threadIdx.x] = s;
}

template <int KIND>
void run(const char* name, float* d) {
    hipEvent_t e0, e1;
    HC(hipEventCreate(&e0));
    HC(hipEventCreate(&e1));
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(rate<KIND>, dim3(256), dim3(1024), 0, 0, d, 3.f);
    HC(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(rate<KIND>, dim3(256), dim3(1024), 0, 0, d, 3.f);
    HC(hipEventRecord(e1));
    HC(hipEventSynchronize(e1));
    float ms;
    HC(hipEventElapsedTime(&ms, e0, e1));
    const double evals = 5.0 * 256 * 16 * ITERS * 8 / 1024.0;  // wave-evaluations per SIMD
    printf("%-58s %8.3f ms  %.3f ns per wave-evaluation per SIMD\n", name, ms / 5, ms * 1e6 / evals);
}

int main() {
    float* d;
    HC(hipMalloc(&d, 256 * 1024 * sizeof(float)));
    run<0>("exp_tab_f32 (shipped: f64, 64-entry double table)", d);
    run<1>("float-float candidate (f32 ops, Ziv test, no fallback)", d);
    run<2>("v_exp_f32 (hardware, inexact: lower bound)", d);
    run<0>("exp_tab_f32 again", d);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
