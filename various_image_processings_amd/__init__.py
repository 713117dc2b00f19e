"""MI355X-native bilateral-filter family (bilateral, joint, adaptive, texture).

A from-scratch gfx950 HIP implementation of the hot path of
yuyuyu-bot/various_image_processings, behind that project's include/cuda API.
The compute runs only in libvip_hip.so (hand-written HIP kernels); this package
is the host-side mirror of the reference interface. See DESIGN.md.
"""
from ._lib import LIB_PATH, VipError, lib  # noqa: F401
from .filters import (  # noqa: F401
    VIP_NUMERICS_CPP,
    VIP_NUMERICS_CUDA,
    CudaAdaptiveBilateralFilter,
    CudaBilateralFilter,
    CudaBilateralTextureFilter,
    DeviceImage,
    cuda_gradient,
    device_synchronize,
    set_bilateral_waves,
)

__version__ = "0.1.0"
