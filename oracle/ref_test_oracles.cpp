// TEST INFRASTRUCTURE ONLY. Never built into, linked by or loaded from the product, and never
// shipped to the GPU box (oracle/_ref/ is git- and gpurun-ignored).
//
// The reference's OWN CPU test oracles, compiled here from /root/reference where they lie.
// oracle/Makefile cuts exactly these line ranges out of the reference's test sources at build
// time (nothing is vendored into this repository, no stand-in header is involved: each range
// uses only the standard headers included below):
//   _ref/ref_adaptive.inc  test/adaptive_bilateral_filter.cu:7-119   RefAdaptiveBilateralFilterImpl
//   _ref/ref_texture.inc   test/bilateral_texture_filter.cu:8-113    RefBilateralTextureFilterImpl
//   _ref/ref_gradient.inc  test/gradient.cu:9-34                     ref_gradient<SrcType>
//   _ref/ref_cpp_luts.inc  include/cpp/bilateral_filter.hpp:10-39   internal::pre_compute_kernels
//                          (the include/cpp filters' space / colour LUTs: double coefficients)
// These are what the reference's gtest suites accept the CUDA kernels against:
// adaptive +-1 (test/adaptive_bilateral_filter.cu:185-193), blur/rtv and gradient FLOAT_EQ
// (test/bilateral_texture_filter.cu:253-262, test/gradient.cu), guide exact EQ
// (test/bilateral_texture_filter.cu:283). tests/golden/make_ref_golden.py calls the C entry
// points below and commits their outputs as tests/golden/ref_oracles.npz.
//
// Built with g++ for x86-64 without -march (the reference's host build: no FMA instructions,
// so no contraction) and -ffp-contract=off to make that explicit.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <memory>
#include <utility>
#include <vector>

#include "_ref/ref_adaptive.inc"
#include "_ref/ref_texture.inc"
#include "_ref/ref_gradient.inc"
#include "_ref/ref_cpp_luts.inc"

extern "C" {

void ref_adaptive(const std::uint8_t* src, std::uint8_t* dst, int width, int height, int ksize, float sigma_space,
                  float sigma_color) {
    RefAdaptiveBilateralFilterImpl impl(width, height, ksize, sigma_space, sigma_color);
    impl.execute(src, dst);
}

void ref_blur_rtv(const std::uint8_t* image, const float* magnitude, float* blurred, float* rtv, int width, int height,
                  int ksize) {
    RefBilateralTextureFilterImpl impl(width, height, ksize);
    impl.compute_blur_and_rtv(image, magnitude, blurred, rtv);
}

void ref_guide(const float* blurred, const float* rtv, std::uint8_t* guide, int width, int height, int ksize) {
    RefBilateralTextureFilterImpl impl(width, height, ksize);
    impl.compute_guide(blurred, rtv, guide);
}

void ref_gradient_u8(const std::uint8_t* src, float* dst, int width, int height, int ch) {
    ref_gradient<std::uint8_t>(src, dst, width, height, ch);
}

void ref_gradient_f32(const float* src, float* dst, int width, int height, int ch) {
    ref_gradient<float>(src, dst, width, height, ch);
}

// include/cpp LUTs: color_len 768 (bilateral, joint: pre_compute_kernels<>) or 1536 (the
// adaptive filter's pre_compute_kernels<512 * 3>); space is ksize x ksize
void ref_cpp_luts(int ksize, float sigma_space, float sigma_color, int color_len, float* space, float* color) {
    auto put = [&](const auto& kv) {
        std::memcpy(space, kv.first.data(), sizeof(float) * kv.first.size());
        std::memcpy(color, kv.second.data(), sizeof(float) * kv.second.size());
    };
    if (color_len == 512 * 3)
        put(internal::pre_compute_kernels<512 * 3>(ksize, sigma_space, sigma_color));
    else
        put(internal::pre_compute_kernels(ksize, sigma_space, sigma_color));
}

}  // extern "C"
