// Shared device/host helpers for the MI355X (gfx950) bilateral-filter family.
// Replaces src/device_utilities.cuh (clamp) and src/host_utilities.hpp
// (CUDASafeCall) of the reference with a status-returning HIP layer.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstdlib>

#include "vip.h"

namespace vip {

// Reference: src/device_utilities.cuh:5-10.
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// static_cast<uint8_t>(v) for v in [0, 256); v_cvt_i32_f32 maps NaN to 0.
__device__ __forceinline__ uint32_t f2u8(float v) { return (uint32_t)(int)v & 0xffu; }

// Round a launch-time size up to a multiple.
constexpr int round_up(int v, int m) { return (v + m - 1) / m * m; }

// Number of LUT copies interleaved in LDS so that the 32 lanes of a ds_read_b32
// half-wave each hit their own bank (bank = (addr/4) % 32): entry d of copy c sits
// at word d*32 + c, so lane l reads word d*32 + (l & 31) -> bank l & 31.
constexpr int kLutCopies = 32;

// Circle half-width of row ky for a disc of radius R: the largest |kx| with
// kx^2 + ky^2 <= R^2 (src/bilateral_filter_impl.cu:222-231 masks the square LUT
// with the same test, so taps outside it carry an exact zero weight).
__host__ __device__ constexpr int isqrt_floor(int v) {
    int r = 0;
    while ((r + 1) * (r + 1) <= v) ++r;
    return r;
}
__host__ __device__ constexpr int circle_hw(int R, int ky) { return isqrt_floor(R * R - ky * ky); }

// Distinct squared tap distances v = kx^2 + ky^2 <= R^2 of the disc (0 <= kx, ky <= R),
// ranked in ascending order: the folded colour x space LUT of the bilateral kernel
// holds one table per distinct v.
__host__ __device__ constexpr bool is_disc_r2(int R, int v) {
    for (int a = 0; a <= R; ++a)
        for (int b = 0; b <= R; ++b)
            if (a * a + b * b == v) return true;
    return false;
}
__host__ __device__ constexpr int disc_r2_rank(int R, int v) {  // distinct disc values below v
    int n = 0;
    for (int u = 0; u < v && u <= R * R; ++u) n += is_disc_r2(R, u) ? 1 : 0;
    return n;
}
__host__ __device__ constexpr int disc_r2_count(int R) { return disc_r2_rank(R, R * R + 1); }

}  // namespace vip

// Record the first error of a call; launch errors come back through
// hipGetLastError (the reference printed them and carried on,
// src/host_utilities.hpp:9-13; the C ABI returns them instead).
#define VIP_HIP_CHECK(expr)                                  \
    do {                                                     \
        hipError_t _e = (expr);                              \
        if (_e != hipSuccess) return (int)_e;                \
    } while (0)

namespace vip {
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per kernel and device (the
// attribute is per device and one process may drive several). `devs` is the
// caller's per-kernel static bitmask; concurrent first calls set it twice, which
// is harmless.
// ABS_LDS: the kernel addresses LDS absolutely (the SatLut tables: a constant byte offset
// in the ds_read immediate), which holds only while its dynamic LDS starts at byte 0, i.e.
// the kernel has no static LDS; checked once, a kernel with any is refused (hipErrorInvalidKernelFile).
inline int ensure_dynamic_lds(const void* kern, int bytes, std::atomic<unsigned long long>& devs,
                              bool abs_lds = false) {
    int dev = 0;
    VIP_HIP_CHECK(hipGetDevice(&dev));
    const unsigned long long bit = 1ull << (dev & 63);
    if (devs.load(std::memory_order_relaxed) & bit) return 0;
    if (abs_lds) {
        hipFuncAttributes fa{};
        VIP_HIP_CHECK(hipFuncGetAttributes(&fa, kern));
        if (fa.sharedSizeBytes != 0) return (int)hipErrorInvalidKernelFile;
    }
    VIP_HIP_CHECK(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    devs.fetch_or(bit, std::memory_order_relaxed);
    return 0;
}

// Launch log of the calling thread (vip_launched_kernels, vip_capi.hip): every stencil and
// texture-stage kernel notes its host stub before its launch, so a caller can name the
// exact template instantiation it timed (bench.py matches it against PMC summaries).
void note_launch(const void* kern);

// Kernel-duration recorder of the calling thread (vip_kernel_timing_*, vip_capi.hip): while
// it is on, the (start, stop) events for the next launch of `kern` on `stream`, else two
// nulls (also for a launch on another device than the recorder's, or into a stream that is
// being captured into a graph: its events would not be stamped).
struct LaunchEvents {
    hipEvent_t start, stop;
};
LaunchEvents timing_events(const void* kern, hipStream_t stream);

// Every stencil and texture launch goes through here: with the recorder on, the launch
// carries an event pair that the runtime stamps with the kernel's own begin and end
// (hipExtLaunchKernel: no marker packet enters the stream, so the duration is the one
// rocprofv3 --kernel-trace reports); otherwise a plain launch.
template <typename K, typename... Args>
inline void launch(K kern, dim3 grid, dim3 block, uint32_t lds, hipStream_t stream, Args... args) {
    const LaunchEvents ev = timing_events(reinterpret_cast<const void*>(kern), stream);
    if (ev.start)
        hipExtLaunchKernelGGL(kern, grid, block, lds, stream, ev.start, ev.stop, 0u, args...);
    else
        hipLaunchKernelGGL(kern, grid, block, lds, stream, args...);
}

// vip_bilateral_set_waves (vip_capi.hip): 0 = per-launch choice, else 16 / 8 / 4.
int bilateral_forced_waves();
// vip_bilateral_set_wide: 0 = per-launch choice, 1 = 128-pixel tiles (8 outputs per
// thread), 2 = 256-pixel tiles (4 outputs per thread, one row per wave).
int bilateral_forced_wide();
}  // namespace vip
