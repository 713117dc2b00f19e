// Drop-in for the reference's include/cuda/device_image.hpp:4-16: a dense
// width*height*channels device buffer with blocking upload/download.
// Backed by vip_malloc / vip_upload / vip_download (hipMalloc + hipMemcpy).
// Unlike the reference (raw owning Impl*, copyable -> double free) the class is
// move-only.
#ifndef VIP_CUDA_DEVICE_IMAGE_HPP
#define VIP_CUDA_DEVICE_IMAGE_HPP

template <typename ElemType>
class DeviceImage {
public:
    DeviceImage(const int width, const int height, const int channels = 1);
    ~DeviceImage();
    DeviceImage(const DeviceImage&) = delete;
    DeviceImage& operator=(const DeviceImage&) = delete;
    DeviceImage(DeviceImage&& other) noexcept;
    DeviceImage& operator=(DeviceImage&& other) noexcept;

    void upload(const ElemType* const data);
    void download(ElemType* const data);
    ElemType* get();

    // Additive stream-ordered copies. `stream` is a hipStream_t
    // passed as void*; the host buffer should be page-locked (vip_host_alloc) for
    // the copy to overlap with kernels on other streams.
    void upload_async(const ElemType* const data, void* stream);
    void download_async(ElemType* const data, void* stream);

private:
    class Impl;
    Impl* impl_;
};

#endif  // VIP_CUDA_DEVICE_IMAGE_HPP
