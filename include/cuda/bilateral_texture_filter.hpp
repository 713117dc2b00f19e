// Drop-in for the reference's include/cuda/bilateral_texture_filter.hpp:7-17.
// Backed by vip_texture_* of include/vip.h. execute() is non-const because the
// object owns its scratch frames; it blocks like the reference (:274).
#ifndef VIP_CUDA_BILATERAL_TEXTURE_FILTER_HPP
#define VIP_CUDA_BILATERAL_TEXTURE_FILTER_HPP

#include <cstdint>
#include <memory>

class CudaBilateralTextureFilter {
public:
    CudaBilateralTextureFilter(const int width, const int height, const int ksize = 9, const int nitr = 3);
    ~CudaBilateralTextureFilter();

    void execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst);
    // additive non-blocking overload: enqueue on `stream` (hipStream_t as void*)
    void execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst, void* stream);

protected:
    class Impl;  // bilateral_texture_filter_impl.cuh
    std::unique_ptr<Impl> impl_;
};

#endif  // VIP_CUDA_BILATERAL_TEXTURE_FILTER_HPP
