// Drop-in for the reference's include/cuda/adaptive_bilateral_filter.hpp:7-24.
// Backed by vip_adaptive_* of include/vip.h; execute() blocks like the reference (:190).
#ifndef VIP_CUDA_ADAPTIVE_BILATERAL_FILTER_HPP
#define VIP_CUDA_ADAPTIVE_BILATERAL_FILTER_HPP

#include <cstdint>
#include <memory>

class CudaAdaptiveBilateralFilter {
public:
    CudaAdaptiveBilateralFilter(const int width, const int height, const int ksize = 9,
                                const float sigma_space = 10.f, const float sigma_color = 30.f);
    ~CudaAdaptiveBilateralFilter();

    void execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst) const;
    // additive non-blocking overload: enqueue on `stream` (hipStream_t as void*)
    void execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst, void* stream) const;

protected:
    class Impl;  // adaptive_bilateral_filter_impl.cuh
    std::unique_ptr<Impl> impl_;
};

#endif  // VIP_CUDA_ADAPTIVE_BILATERAL_FILTER_HPP
