// The joint filter's source plane as f16 (round 5): a tap's accumulation would read the
// source channel as an f16 and fuse it into v_fma_mix_f32 instead of converting the byte
// with v_cvt_f32_ubyteN and using v_fma_f32. Bit-exact only if
//   fma_mix(w, (f16)b, acc) == fmaf(w, (float)b, acc)
// for every byte b, every weight w the folded tables hold (denormals included) and every
// accumulator. Part 1 checks that over random and edge bit patterns (the f16 of a byte is
// exact, so only the fused rounding and the denormal handling can differ). Part 2 times
// v_fma_mix_f32 against v_fma_f32 (16 waves per CU, 8 independent chains per lane; the
// byte conversion it would remove costs one slow-class VALU, profiles/r02_valu_rates.txt).
#include <hip/hip_runtime.h>

#include <cstdint>
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

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// one case per thread: w from a bit pattern (every class: denormal, normal, tiny, 1),
// b a byte, acc a non-negative float of the accumulator's range or a random pattern
__global__ void check(const _Float16* h16, unsigned long long* bad, uint32_t seed, uint32_t* example) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const uint32_t r0 = hash(i * 3u + seed), r1 = hash(i * 3u + 1u + seed), r2 = hash(i * 3u + 2u + seed);
    uint32_t wb;
    switch (r0 & 3u) {
        case 0: wb = r1 & 0x007fffffu; break;                       // denormal
        case 1: wb = (r1 & 0x3f7fffffu); break;                     // (0, 1)
        case 2: wb = 0x00800000u + (r1 & 0x03ffffffu); break;       // small normal
        default: wb = r1 & 0x7f7fffffu; break;                      // any finite >= 0
    }
    const float w = __builtin_bit_cast(float, wb);
    const uint32_t b = (r0 >> 8) & 255u;
    float acc;
    if ((r0 >> 16) & 1u) acc = (float)(r2 % 12495u) + __builtin_bit_cast(float, 0x3f000000u | (r2 >> 9)) - 0.5f;
    else acc = __builtin_bit_cast(float, r2 & 0x7f7fffffu);
    if ((r0 >> 17) & 1u) acc = __builtin_bit_cast(float, r2 & 0x007fffffu);  // denormal accumulator
    const float want = __builtin_fmaf(w, (float)b, acc);                 // v_cvt_f32_ubyte0 + v_fma_f32
    const float got = __builtin_fmaf(w, (float)h16[b], acc);             // v_fma_mix_f32
    if (__builtin_bit_cast(uint32_t, want) != __builtin_bit_cast(uint32_t, got)) {
        if (atomicAdd(bad, 1ull) == 0ull) {
            example[0] = wb; example[1] = b; example[2] = __builtin_bit_cast(uint32_t, acc);
            example[3] = __builtin_bit_cast(uint32_t, want); example[4] = __builtin_bit_cast(uint32_t, got);
        }
    }
}

#define ITERS 4096
template <bool MIX>
__global__ __launch_bounds__(1024) void rate(float* out, const _Float16* h16, float seed) {
    float acc[8];
    uint32_t hv[8];  // an f16 in the low half (opaque per iteration: no hoisted conversion)
    float fv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        acc[i] = seed * i;
        hv[i] = __builtin_bit_cast(uint16_t, h16[(threadIdx.x + i) & 255]);
        fv[i] = (float)((threadIdx.x * 7u + i) & 255u);
    }
    const float w = seed * 1e-3f;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (MIX) {
                __asm__ volatile("" : "+v"(hv[i]));
                acc[i] = __builtin_fmaf(w, (float)__builtin_bit_cast(_Float16, (uint16_t)hv[i]), acc[i]);
            } else {
                __asm__ volatile("" : "+v"(fv[i]));
                acc[i] = __builtin_fmaf(w, fv[i], acc[i]);
            }
        }
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += acc[i];
    out[blockIdx.x * 1024 + threadIdx.x] = s;
}

template <bool MIX>
void run(const char* name, float* d, const _Float16* h16) {
    hipEvent_t e0, e1;
    HC(hipEventCreate(&e0));
    HC(hipEventCreate(&e1));
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(rate<MIX>, dim3(256), dim3(1024), 0, 0, d, h16, 3.f);
    HC(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(rate<MIX>, dim3(256), dim3(1024), 0, 0, d, h16, 3.f);
    HC(hipEventRecord(e1));
    HC(hipEventSynchronize(e1));
    float ms;
    HC(hipEventElapsedTime(&ms, e0, e1));
    const double n = 5.0 * 256 * 16 * ITERS * 8 / 1024.0;  // wave-FMAs per SIMD
    printf("%-44s %8.3f ms  %.3f ns per wave-FMA per SIMD\n", name, ms / 5, ms * 1e6 / n);
}

int main() {
    _Float16 hh[256];
    for (int b = 0; b < 256; ++b) hh[b] = (_Float16)b;
    _Float16* h16;
    unsigned long long* bad;
    uint32_t* ex;
    float* d;
    HC(hipMalloc(&h16, sizeof hh));
    HC(hipMemcpy(h16, hh, sizeof hh, hipMemcpyHostToDevice));
    HC(hipMalloc(&bad, sizeof(unsigned long long)));
    HC(hipMemset(bad, 0, sizeof(unsigned long long)));
    HC(hipMalloc(&ex, 5 * sizeof(uint32_t)));
    HC(hipMalloc(&d, 256 * 1024 * sizeof(float)));
    const uint32_t per = 1u << 24;
    for (uint32_t s = 0; s < 64; ++s) hipLaunchKernelGGL(check, dim3(per / 256), dim3(256), 0, 0, h16, bad, s * per * 3u, ex);
    HC(hipDeviceSynchronize());
    unsigned long long nb = 0;
    uint32_t e[5] = {};
    HC(hipMemcpy(&nb, bad, sizeof nb, hipMemcpyDeviceToHost));
    HC(hipMemcpy(e, ex, sizeof e, hipMemcpyDeviceToHost));
    printf("fma_mix(w, (f16)b, acc) vs fmaf(w, (float)b, acc): %llu mismatches in %u cases\n", nb, 64u * per);
    if (nb) printf("  first: w %08x b %u acc %08x want %08x got %08x\n", e[0], e[1], e[2], e[3], e[4]);
    run<false>("v_fma_f32 (f32 operand)", d, h16);
    run<true>("v_fma_mix_f32 (f16 operand)", d, h16);
    run<false>("v_fma_f32 again", d, h16);
    return nb == 0 ? 0 : 2;
}
