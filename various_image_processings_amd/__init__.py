"""MI355X-native bilateral-filter family (bilateral, joint, adaptive, texture).

A from-scratch gfx950 HIP implementation of the hot path of
yuyuyu-bot/various_image_processings, behind that project's include/cuda API.
The compute runs only in libvip_hip.so (hand-written HIP kernels); this package
is the host-side mirror of the reference interface. See DESIGN.md.
"""
from ._lib import (  # noqa: F401
    LIB_PATH,
    VIP_FILTER_ADAPTIVE,
    VIP_FILTER_BILATERAL,
    VIP_FILTER_JOINT,
    VIP_FILTER_TEXTURE,
    VIP_PATH_AUTO,
    VIP_PATH_RUNTIME,
    VipError,
    lib,
)
from .filters import (  # noqa: F401
    VIP_NUMERICS_CPP,
    VIP_NUMERICS_CUDA,
    CudaAdaptiveBilateralFilter,
    CudaBilateralFilter,
    CudaBilateralTextureFilter,
    DeviceImage,
    cuda_gradient,
    device_synchronize,
    kernel_timing,
    launched_kernels,
    max_ksize,
    set_bilateral_frames_in_flight,
    set_bilateral_waves,
    set_bilateral_wide,
    set_stencil_path,
)

__version__ = "0.1.0"
