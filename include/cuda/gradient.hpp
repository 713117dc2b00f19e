// Drop-in for the reference's include/cuda/gradient.hpp:4-23: central-difference
// gradient magnitude of a dense u8 or f32 image with src_ch in {1, 3}, into a
// dense f32 image. Backed by vip_gradient_u8 / vip_gradient_f32 (include/vip.h).
// Like the reference (src/gradient_impl.cu:90-103) the call does not synchronise.
#ifndef VIP_CUDA_GRADIENT_HPP
#define VIP_CUDA_GRADIENT_HPP

#include <cstdint>
#include <type_traits>

template <typename SrcType>
void cuda_gradient_impl(const SrcType* const d_src, float* const d_dst, const int width, const int height,
                        const int src_ch);

template <typename SrcType>
void cuda_gradient(const SrcType* const d_src, float* const d_dst, const int width, const int height,
                   const int src_ch = 1) {
    static_assert(std::is_same_v<SrcType, std::uint8_t> || std::is_same_v<SrcType, float>,
                  "cuda_gradient supports uint8_t and float sources");
    cuda_gradient_impl(d_src, d_dst, width, height, src_ch);
}

#endif  // VIP_CUDA_GRADIENT_HPP
