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

    void upload(const ElemType* const data);
    void download(ElemType* const data);
    ElemType* get();

private:
    class Impl;
    Impl* impl_;
};

#endif  // VIP_CUDA_DEVICE_IMAGE_HPP
