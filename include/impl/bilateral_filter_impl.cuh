// Impl of CudaBilateralFilter, visible to test drivers the way the reference's
// src/bilateral_filter_impl.cuh:7-33 is (test/bilateral_filter.cu:9-33 subclasses
// the public class and calls impl_->bilateral_filter without a device sync).
// Methods here are asynchronous on the default stream.
#ifndef VIP_IMPL_BILATERAL_FILTER_IMPL_CUH
#define VIP_IMPL_BILATERAL_FILTER_IMPL_CUH

#include <cstdint>

#include "cuda/bilateral_filter.hpp"
#include "vip.h"

class CudaBilateralFilter::Impl {
public:
    Impl(const int width, const int height, const int ksize = 9, const float sigma_space = 10.f,
         const float sigma_color = 30.f);
    ~Impl();
    Impl(const Impl&) = delete;
    Impl& operator=(const Impl&) = delete;

    void bilateral_filter(const std::uint8_t* const d_src, std::uint8_t* const d_dst) const;
    void joint_bilateral_filter(const std::uint8_t* const d_src, const std::uint8_t* const d_guide,
                                std::uint8_t* const d_dst) const;
    void bilateral_filter(const std::uint8_t* const d_src, std::uint8_t* const d_dst, void* stream) const;
    void joint_bilateral_filter(const std::uint8_t* const d_src, const std::uint8_t* const d_guide,
                                std::uint8_t* const d_dst, void* stream) const;

    vip_bilateral_t handle() const { return handle_; }

private:
    const int width_;
    vip_bilateral_t handle_ = nullptr;
};

#endif  // VIP_IMPL_BILATERAL_FILTER_IMPL_CUH
