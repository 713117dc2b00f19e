// Exactness check of the bilateral epilogue's division (vip_stencil.hpp div_by_sumk):
//   y  = rcp(k) refined by one Newton step          -- must equal RN(1/k)
//   q0 = RN(s * y); r = fma(-k, q0, s); q = fma(r, y, q0)  -- must equal RN(s / k)
// (a) the reciprocal EXHAUSTIVELY for every float k in [1, 2^38) -- the sum of
//     weights of a bilateral/joint window (the centre tap weighs exactly 1, every
//     tap at most 1, at most 31*31 taps) and the texture guide's 1 + exp(x) in
//     [2, 1 + e^25.5] (x = sigma_alpha (rtv - rtv_min) <= 255 / (5 ksize): up to 2^37 at
//     ksize 2);
// (b) the quotient for 2^30 pseudo-random (s, k), s in [0, 255 k], and for s at the
//     float midpoints' neighbourhoods -- Markstein's theorem makes (b) follow from (a),
//     this is the empirical cross-check.
// (c) vip::sqrt_int_exact against sqrtf for every integer in [0, 2^20) (texture gradient).
// (d) vip::pack_u8_clamped against clampi((int)v, 0, 255) for every float |v| < 2048 (the
//     texture guide's blend: v in [-255, 511]).
// (e) vip::exp_tab_f32 against (float)exp((double)x) (ocml's double exp) for every float x
//     in [0, 32) (the texture guide's alpha argument lies in [0, 25.5]).
// (f) vip::rtv_quotient(n, d) against (float)(n / d) for 2^30 pseudo-random inputs: half
//     the guide stage's own (n a float in [0, 2^18), d = (double)msum + 1e-9 with msum a
//     float in [0, 2^19)), half with n / d placed within +-80 double ulps of a float
//     rounding midpoint (the fallback's territory).
// Exit status 0 iff no mismatch against the IEEE divide / sqrt (hipcc default, correctly
// rounded). Run on the GPU: tests/test_gpu_parity.py::test_epilogue_division_exact.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "vip_stencil.hpp"

__device__ unsigned long long g_bad[6];
__device__ unsigned int g_exp_bad_x[16];

__global__ void exp_all(uint32_t n) {
    __shared__ double etab[64];
    if (threadIdx.x < 64) etab[threadIdx.x] = vip::kExp2Tab64[threadIdx.x];
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = __uint_as_float(i);
    const float want = (float)exp((double)x);
    if (__float_as_uint(vip::exp_tab_f32(x, etab)) != __float_as_uint(want)) {
        const unsigned long long slot = atomicAdd(&g_bad[4], 1ull);
        if (slot < 16) g_exp_bad_x[slot] = i;
    }
}

// (d) every float with |v| < 2048: both signs of the bit patterns [0, 0x45000000)
__global__ void pack_u8_all(uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
#pragma unroll
    for (uint32_t sign = 0; sign < 2; ++sign) {
        const float v = __uint_as_float((sign << 31) | i);
        const uint32_t want = (uint32_t)vip::clampi((int)v, 0, 255) << 16 | 0xa5005aa5u;  // byte 2 replaced
        if (vip::pack_u8_clamped(v, 2, 0xa5a55aa5u) != want) atomicAdd(&g_bad[3], 1ull);
    }
}

// (c) the texture gradient's integer square root: vip::sqrt_int_exact == sqrtf (hipcc's
//     correctly rounded expansion) for every integer in [0, n)
__global__ void sqrt_ints(uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = (float)i;
    if (__float_as_uint(vip::sqrt_int_exact(x)) != __float_as_uint(__builtin_sqrtf(x))) atomicAdd(&g_bad[2], 1ull);
}

__global__ void recip_all(uint32_t lo_bits, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float k = __uint_as_float(lo_bits + i);
    const float y = vip::recip_exact(k);
    const float want = 1.0f / k;  // IEEE, correctly rounded
    if (__float_as_uint(y) != __float_as_uint(want)) atomicAdd(&g_bad[0], 1ull);
}

__device__ __forceinline__ uint32_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return (uint32_t)x;
}

__global__ void quot_random(uint64_t base) {
    const uint64_t i = base + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint32_t a = mix(2 * i), b = mix(2 * i + 1);
    const float k = 1.0f + (float)(a >> 9) * (1023.0f / 8388608.0f);  // [1, 1024)
    float s;
    if (b & 1) {
        s = (float)(b >> 8) * (255.0f / 16777216.0f) * k;  // uniform in [0, 255 k)
    } else {
        // near a float midpoint of the quotient: s = k * (m + half ulp) +- a few ulp
        const float m = (float)(b >> 9) * (255.0f / 8388608.0f);
        const float mid = m + 0.5f * (__uint_as_float(__float_as_uint(m) + 1) - m);
        s = __uint_as_float(__float_as_uint(mid * k) + (int)(b >> 28) - 8);
    }
    const float y = vip::recip_exact(k);
    const float q = vip::div_by_sumk(s, k, y);
    const float want = s / k;
    if (__float_as_uint(q) != __float_as_uint(want)) atomicAdd(&g_bad[1], 1ull);
}

__global__ void rtv_random(uint64_t base) {
    const uint64_t i = base + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint32_t a = mix(3 * i), b = mix(3 * i + 1), c = mix(3 * i + 2);
    const float msum = __uint_as_float(a & 0x7fffffffu) < 524288.0f ? __uint_as_float(a & 0x7fffffffu)
                                                                      : (float)(a >> 13);  // [0, 2^19)
    const double d = (double)msum + 1e-9;
    double n;
    if (c & 1) {
        n = (double)((float)(b >> 14) + (float)(b & 0x3fff) * (1.0f / 16384.0f));  // a float in [0, 2^18)
    } else {
        // n / d within +-80 double ulps of the midpoint between float m and its successor
        const float m = (float)(b >> 9) * (1.0f / 64.0f) + __uint_as_float(0x38000000u);
        const double mid = 0.5 * ((double)m + (double)__uint_as_float(__float_as_uint(m) + 1));
        const double t = __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, mid) + (long long)(c >> 24) - 80);
        n = t * d;
    }
    if (__float_as_uint(vip::rtv_quotient(n, d)) != __float_as_uint((float)(n / d))) atomicAdd(&g_bad[5], 1ull);
}

int main() {
    unsigned long long zero[6] = {0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_bad), zero, sizeof(zero)) != hipSuccess) return 2;
    // bit patterns of 1.0f and 2^38: the epilogue's sums of weights lie in [1, 1024), the
    // texture guide's 1 + exp(x) in [2, 2^37) (x <= 25.5 at ksize 2)
    const uint32_t lo = 0x3f800000u, hi = 0x52800000u;
    const uint32_t n = hi - lo;
    hipLaunchKernelGGL(recip_all, dim3((n + 255) / 256), dim3(256), 0, 0, lo, n);
    const uint64_t per = 1ull << 26;
    for (int rep = 0; rep < 16; ++rep)
        hipLaunchKernelGGL(quot_random, dim3((unsigned)(per / 256)), dim3(256), 0, 0, rep * per);
    const uint32_t nsq = 1u << 20;
    hipLaunchKernelGGL(sqrt_ints, dim3(nsq / 256), dim3(256), 0, 0, nsq);
    const uint32_t npk = 0x45000000u;
    hipLaunchKernelGGL(pack_u8_all, dim3((npk + 255) / 256), dim3(256), 0, 0, npk);
    const uint32_t nexp = 0x42000000u;  // bit patterns of [0, 32)
    hipLaunchKernelGGL(exp_all, dim3((nexp + 255) / 256), dim3(256), 0, 0, nexp);
    for (int rep = 0; rep < 16; ++rep)
        hipLaunchKernelGGL(rtv_random, dim3((unsigned)(per / 256)), dim3(256), 0, 0, rep * per);
    unsigned long long bad[6];
    if (hipMemcpyFromSymbol(bad, HIP_SYMBOL(g_bad), sizeof(bad)) != hipSuccess) return 2;
    std::printf("reciprocal: %u floats k in [1, 2^38), %llu mismatches\n", n, bad[0]);
    std::printf("quotient: %llu random (s, k), %llu mismatches\n", (unsigned long long)(16 * per), bad[1]);
    std::printf("integer sqrt: %u integers in [0, 2^20), %llu mismatches\n", nsq, bad[2]);
    std::printf("u8 clamp pack: %u floats |v| < 2048 of each sign, %llu mismatches\n", npk, bad[3]);
    std::printf("exp: %u floats x in [0, 32), %llu mismatches\n", nexp, bad[4]);
    std::printf("rtv quotient: %llu random (n, d), half at float midpoints, %llu mismatches\n",
                (unsigned long long)(16 * per), bad[5]);
    if (bad[4]) {
        unsigned int xs[16];
        if (hipMemcpyFromSymbol(xs, HIP_SYMBOL(g_exp_bad_x), sizeof(xs)) == hipSuccess)
            for (unsigned long long j = 0; j < bad[4] && j < 16; ++j) std::printf("  exp mismatch at x = %a\n", (double)__builtin_bit_cast(float, xs[j]));
    }
    return (bad[0] || bad[1] || bad[2] || bad[3] || bad[4] || bad[5]) ? 1 : 0;
}
