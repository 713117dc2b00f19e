// Impl of CudaBilateralTextureFilter (reference: src/bilateral_texture_filter_impl.cuh:7-45).
// test/bilateral_texture_filter.cu:115-136 drives the two stages through
// thrust::device_vector references; those overloads are inline and compiled only
// when a thrust implementation (rocThrust on ROCm) is on the include path, so the
// library itself has no thrust dependency.
#ifndef VIP_IMPL_BILATERAL_TEXTURE_FILTER_IMPL_CUH
#define VIP_IMPL_BILATERAL_TEXTURE_FILTER_IMPL_CUH

#include <cstdint>

#include "cuda/bilateral_texture_filter.hpp"
#include "vip.h"

#if defined(__has_include)
#if __has_include(<thrust/device_vector.h>) && defined(__HIPCC__)
#include <thrust/device_vector.h>
#define VIP_HAVE_THRUST 1
#endif
#endif

class CudaBilateralTextureFilter::Impl {
public:
    Impl(const int width, const int height, const int ksize = 9, const int nitr = 3);
    ~Impl();
    Impl(const Impl&) = delete;
    Impl& operator=(const Impl&) = delete;

    void execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst);
    void execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst, void* stream);

    // stage entry points (no synchronisation), raw device pointers
    void compute_blur_and_rtv(const std::uint8_t* d_image, const float* d_magnitude, float* d_blurred, float* d_rtv);
    void compute_guide(const float* d_blurred, const float* d_rtv, std::uint8_t* d_guide);

#ifdef VIP_HAVE_THRUST
    void compute_blur_and_rtv(const thrust::device_vector<std::uint8_t>& d_image,
                              const thrust::device_vector<float>& d_magnitude, thrust::device_vector<float>& d_blurred,
                              thrust::device_vector<float>& d_rtv) {
        compute_blur_and_rtv(d_image.data().get(), d_magnitude.data().get(), d_blurred.data().get(),
                             d_rtv.data().get());
    }
    void compute_guide(const thrust::device_vector<float>& d_blurred, const thrust::device_vector<float>& d_rtv,
                       thrust::device_vector<std::uint8_t>& d_guide) {
        compute_guide(d_blurred.data().get(), d_rtv.data().get(), d_guide.data().get());
    }
#endif

    vip_texture_t handle() const { return handle_; }

private:
    vip_texture_t handle_ = nullptr;
};

#endif  // VIP_IMPL_BILATERAL_TEXTURE_FILTER_IMPL_CUH
