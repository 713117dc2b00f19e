// Drop-in for the reference's include/cuda/bilateral_filter.hpp:7-29.
// Same class name, constructor defaults and member signatures, so
// sample/bilateral_filter/main.cpp and test/bilateral_filter.cu compile against it.
// Backed by the C ABI in include/vip.h (libvip_hip.so, gfx950 HIP kernels).
// Pointers are device pointers to dense width*3 uint8 images; public calls block
// until the GPU is done (the reference synchronised the device, :299, :309).
#ifndef VIP_CUDA_BILATERAL_FILTER_HPP
#define VIP_CUDA_BILATERAL_FILTER_HPP

#include <cstdint>
#include <memory>

class CudaBilateralFilter {
public:
    CudaBilateralFilter(const int width, const int height, const int ksize = 9, const float sigma_space = 10.f,
                        const float sigma_color = 30.f);
    ~CudaBilateralFilter();

    void bilateral_filter(const std::uint8_t* const d_src, std::uint8_t* const d_dst) const;

    void joint_bilateral_filter(const std::uint8_t* const d_src, const std::uint8_t* const d_guide,
                                std::uint8_t* const d_dst) const;

    // Additive, non-blocking overloads: enqueue on `stream` (a
    // hipStream_t passed as void*, nullptr = default stream) and return at once.
    void bilateral_filter(const std::uint8_t* const d_src, std::uint8_t* const d_dst, void* stream) const;
    void joint_bilateral_filter(const std::uint8_t* const d_src, const std::uint8_t* const d_guide,
                                std::uint8_t* const d_dst, void* stream) const;

protected:
    class Impl;  // defined in bilateral_filter_impl.cuh (test drivers reach it through impl_)
    std::unique_ptr<Impl> impl_;
};

#endif  // VIP_CUDA_BILATERAL_FILTER_HPP
