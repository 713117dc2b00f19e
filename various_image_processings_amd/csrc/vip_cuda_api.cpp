// C++ drop-in API (include/cuda/*.hpp + include/impl/*.cuh) implemented over the
// C ABI. Error behaviour follows the reference's CUDASafeCall
// (src/host_utilities.hpp:9-13): print "HIP Error <file> : <line> <message>" to
// stderr and carry on; allocation failures in constructors throw
// std::runtime_error (thrust::device_vector threw std::bad_alloc in the reference).


#include <cstdio>
#include <stdexcept>
#include <string>

#include "cuda/device_image.hpp"
#include "cuda/gradient.hpp"
#include "impl/adaptive_bilateral_filter_impl.cuh"
#include "impl/bilateral_filter_impl.cuh"
#include "impl/bilateral_texture_filter_impl.cuh"
#include "vip.h"

namespace {

void report(int rc, const char* file, int line) {
    if (rc != 0) std::fprintf(stderr, "HIP Error %s : %d %s\n", file, line, vip_error_string(rc));
}
#define VIP_REPORT(expr) report((expr), __FILE__, __LINE__)

[[noreturn]] void fail(const char* what, int rc) {
    throw std::runtime_error(std::string(what) + ": " + vip_error_string(rc));
}

}  // namespace

// ------------------------------------------------------------ CudaBilateralFilter
CudaBilateralFilter::Impl::Impl(const int width, const int height, const int ksize, const float sigma_space,
                                const float sigma_color)
    : width_(width) {
    (void)height;
    const int rc = vip_bilateral_create(&handle_, width, height, ksize, sigma_space, sigma_color, VIP_NUMERICS_CUDA);
    if (rc) fail("CudaBilateralFilter", rc);
}
CudaBilateralFilter::Impl::~Impl() { vip_bilateral_destroy(handle_); }

void CudaBilateralFilter::Impl::bilateral_filter(const std::uint8_t* const d_src, std::uint8_t* const d_dst) const {
    bilateral_filter(d_src, d_dst, nullptr);
}
void CudaBilateralFilter::Impl::bilateral_filter(const std::uint8_t* const d_src, std::uint8_t* const d_dst,
                                                 void* stream) const {
    VIP_REPORT(vip_bilateral_run(handle_, d_src, (size_t)width_ * 3, d_dst, (size_t)width_ * 3, stream));
}

void CudaBilateralFilter::Impl::joint_bilateral_filter(const std::uint8_t* const d_src,
                                                       const std::uint8_t* const d_guide,
                                                       std::uint8_t* const d_dst) const {
    joint_bilateral_filter(d_src, d_guide, d_dst, nullptr);
}
void CudaBilateralFilter::Impl::joint_bilateral_filter(const std::uint8_t* const d_src,
                                                       const std::uint8_t* const d_guide, std::uint8_t* const d_dst,
                                                       void* stream) const {
    const size_t pitch = (size_t)width_ * 3;
    VIP_REPORT(vip_joint_bilateral_run(handle_, d_src, pitch, d_guide, pitch, d_dst, pitch, stream));
}

CudaBilateralFilter::CudaBilateralFilter(const int width, const int height, const int ksize, const float sigma_space,
                                         const float sigma_color)
    : impl_(std::make_unique<Impl>(width, height, ksize, sigma_space, sigma_color)) {}
CudaBilateralFilter::~CudaBilateralFilter() = default;

void CudaBilateralFilter::bilateral_filter(const std::uint8_t* const d_src, std::uint8_t* const d_dst) const {
    impl_->bilateral_filter(d_src, d_dst);
    VIP_REPORT(vip_device_synchronize());
}

void CudaBilateralFilter::joint_bilateral_filter(const std::uint8_t* const d_src, const std::uint8_t* const d_guide,
                                                 std::uint8_t* const d_dst) const {
    impl_->joint_bilateral_filter(d_src, d_guide, d_dst);
    VIP_REPORT(vip_device_synchronize());
}

void CudaBilateralFilter::bilateral_filter(const std::uint8_t* const d_src, std::uint8_t* const d_dst,
                                           void* stream) const {
    impl_->bilateral_filter(d_src, d_dst, stream);
}

void CudaBilateralFilter::joint_bilateral_filter(const std::uint8_t* const d_src, const std::uint8_t* const d_guide,
                                                 std::uint8_t* const d_dst, void* stream) const {
    impl_->joint_bilateral_filter(d_src, d_guide, d_dst, stream);
}

// ------------------------------------------------------------ CudaAdaptiveBilateralFilter
CudaAdaptiveBilateralFilter::Impl::Impl(const int width, const int height, const int ksize, const float sigma_space,
                                        const float sigma_color)
    : width_(width) {
    (void)height;
    const int rc = vip_adaptive_create(&handle_, width, height, ksize, sigma_space, sigma_color, VIP_NUMERICS_CUDA);
    if (rc) fail("CudaAdaptiveBilateralFilter", rc);
}
CudaAdaptiveBilateralFilter::Impl::~Impl() { vip_adaptive_destroy(handle_); }

void CudaAdaptiveBilateralFilter::Impl::execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst) const {
    execute(d_src, d_dst, nullptr);
}
void CudaAdaptiveBilateralFilter::Impl::execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst,
                                                void* stream) const {
    VIP_REPORT(vip_adaptive_run(handle_, d_src, (size_t)width_ * 3, d_dst, (size_t)width_ * 3, stream));
}

CudaAdaptiveBilateralFilter::CudaAdaptiveBilateralFilter(const int width, const int height, const int ksize,
                                                         const float sigma_space, const float sigma_color)
    : impl_(std::make_unique<Impl>(width, height, ksize, sigma_space, sigma_color)) {}
CudaAdaptiveBilateralFilter::~CudaAdaptiveBilateralFilter() = default;

void CudaAdaptiveBilateralFilter::execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst) const {
    impl_->execute(d_src, d_dst);
    VIP_REPORT(vip_device_synchronize());
}

void CudaAdaptiveBilateralFilter::execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst,
                                          void* stream) const {
    impl_->execute(d_src, d_dst, stream);
}

// ------------------------------------------------------------ CudaBilateralTextureFilter
CudaBilateralTextureFilter::Impl::Impl(const int width, const int height, const int ksize, const int nitr) {
    const int rc = vip_texture_create(&handle_, width, height, ksize, nitr, VIP_NUMERICS_CUDA);
    if (rc) fail("CudaBilateralTextureFilter", rc);
}
CudaBilateralTextureFilter::Impl::~Impl() { vip_texture_destroy(handle_); }

void CudaBilateralTextureFilter::Impl::execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst) {
    execute(d_src, d_dst, nullptr);
}
void CudaBilateralTextureFilter::Impl::execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst,
                                               void* stream) {
    VIP_REPORT(vip_texture_run(handle_, d_src, d_dst, stream));
}

void CudaBilateralTextureFilter::Impl::compute_blur_and_rtv(const std::uint8_t* d_image, const float* d_magnitude,
                                                            float* d_blurred, float* d_rtv) {
    VIP_REPORT(vip_texture_blur_rtv(handle_, d_image, d_magnitude, d_blurred, d_rtv, nullptr));
}

void CudaBilateralTextureFilter::Impl::compute_guide(const float* d_blurred, const float* d_rtv,
                                                     std::uint8_t* d_guide) {
    VIP_REPORT(vip_texture_guide(handle_, d_blurred, d_rtv, d_guide, nullptr));
}

CudaBilateralTextureFilter::CudaBilateralTextureFilter(const int width, const int height, const int ksize,
                                                       const int nitr)
    : impl_(std::make_unique<Impl>(width, height, ksize, nitr)) {}
CudaBilateralTextureFilter::~CudaBilateralTextureFilter() = default;

void CudaBilateralTextureFilter::execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst) {
    impl_->execute(d_src, d_dst);
    VIP_REPORT(vip_device_synchronize());
}

void CudaBilateralTextureFilter::execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst, void* stream) {
    impl_->execute(d_src, d_dst, stream);
}

// ------------------------------------------------------------ cuda_gradient
template <>
void cuda_gradient_impl<std::uint8_t>(const std::uint8_t* const d_src, float* const d_dst, const int width,
                                      const int height, const int src_ch) {
    VIP_REPORT(vip_gradient_u8(d_src, d_dst, width, height, src_ch, VIP_NUMERICS_CUDA, nullptr));
}

template <>
void cuda_gradient_impl<float>(const float* const d_src, float* const d_dst, const int width, const int height,
                               const int src_ch) {
    VIP_REPORT(vip_gradient_f32(d_src, d_dst, width, height, src_ch, VIP_NUMERICS_CUDA, nullptr));
}

// ------------------------------------------------------------ DeviceImage
template <typename ElemType>
class DeviceImage<ElemType>::Impl {
public:
    explicit Impl(const size_t len) : len_(len) {
        const int rc = vip_malloc(reinterpret_cast<void**>(&data_), len * sizeof(ElemType));
        if (rc) fail("DeviceImage", rc);
    }
    ~Impl() { vip_free(data_); }
    void upload(const ElemType* const data) { VIP_REPORT(vip_upload(data_, data, len_ * sizeof(ElemType))); }
    void download(ElemType* const data) { VIP_REPORT(vip_download(data, data_, len_ * sizeof(ElemType))); }
    void upload_async(const ElemType* const data, void* stream) {
        VIP_REPORT(vip_upload_async(data_, data, len_ * sizeof(ElemType), stream));
    }
    void download_async(ElemType* const data, void* stream) {
        VIP_REPORT(vip_download_async(data, data_, len_ * sizeof(ElemType), stream));
    }
    ElemType* get() { return data_; }

private:
    size_t len_;
    ElemType* data_ = nullptr;
};

template <typename ElemType>
DeviceImage<ElemType>::DeviceImage(const int width, const int height, const int channels)
    : impl_(new Impl((size_t)width * height * channels)) {}

template <typename ElemType>
DeviceImage<ElemType>::~DeviceImage() {
    delete impl_;
}

template <typename ElemType>
DeviceImage<ElemType>::DeviceImage(DeviceImage&& other) noexcept : impl_(other.impl_) {
    other.impl_ = nullptr;
}

template <typename ElemType>
DeviceImage<ElemType>& DeviceImage<ElemType>::operator=(DeviceImage&& other) noexcept {
    if (this != &other) {
        delete impl_;
        impl_ = other.impl_;
        other.impl_ = nullptr;
    }
    return *this;
}

template <typename ElemType>
void DeviceImage<ElemType>::upload(const ElemType* const data) {
    impl_->upload(data);
}

template <typename ElemType>
void DeviceImage<ElemType>::download(ElemType* const data) {
    impl_->download(data);
}

template <typename ElemType>
ElemType* DeviceImage<ElemType>::get() {
    return impl_->get();
}

template <typename ElemType>
void DeviceImage<ElemType>::upload_async(const ElemType* const data, void* stream) {
    impl_->upload_async(data, stream);
}

template <typename ElemType>
void DeviceImage<ElemType>::download_async(ElemType* const data, void* stream) {
    impl_->download_async(data, stream);
}

template class DeviceImage<std::uint8_t>;
template class DeviceImage<float>;
