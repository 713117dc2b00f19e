// Impl of CudaAdaptiveBilateralFilter (reference: src/adaptive_bilateral_filter_impl.cuh:7-29,
// reached by test/adaptive_bilateral_filter.cu:121-137). execute() here does not synchronise.
#ifndef VIP_IMPL_ADAPTIVE_BILATERAL_FILTER_IMPL_CUH
#define VIP_IMPL_ADAPTIVE_BILATERAL_FILTER_IMPL_CUH

#include <cstdint>

#include "cuda/adaptive_bilateral_filter.hpp"
#include "vip.h"

class CudaAdaptiveBilateralFilter::Impl {
public:
    Impl(const int width, const int height, const int ksize = 9, const float sigma_space = 10.f,
         const float sigma_color = 30.f);
    ~Impl();
    Impl(const Impl&) = delete;
    Impl& operator=(const Impl&) = delete;

    void execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst) const;
    void execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst, void* stream) const;

    vip_adaptive_t handle() const { return handle_; }

private:
    const int width_;
    vip_adaptive_t handle_ = nullptr;
};

#endif  // VIP_IMPL_ADAPTIVE_BILATERAL_FILTER_IMPL_CUH
