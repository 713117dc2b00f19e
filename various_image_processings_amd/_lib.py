"""ctypes binding of the C ABI in include/vip.h (libvip_hip.so, gfx950 HIP kernels).

The shared library is built in-tree by ``__graft_entry__.build()`` (``make -C
various_image_processings_amd/csrc``). There is no fallback: if the library is
missing or cannot be loaded, :func:`lib` raises, so no caller can silently run
anything but the HIP kernels.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libvip_hip.so")

VIP_NUMERICS_CUDA = 0
VIP_NUMERICS_CPP = 1
VIP_ERR_INVALID_ARGUMENT = 10001
VIP_ERR_UNSUPPORTED_KSIZE = 10002
VIP_ERR_ALIASING = 10003
VIP_FILTER_BILATERAL, VIP_FILTER_JOINT, VIP_FILTER_ADAPTIVE, VIP_FILTER_TEXTURE = 0, 1, 2, 3
VIP_PATH_AUTO, VIP_PATH_RUNTIME = 0, 1

_c_void_p = ctypes.c_void_p
_c_int = ctypes.c_int
_c_float = ctypes.c_float
_c_size_t = ctypes.c_size_t

# name -> (restype, argtypes); every entry point declared in include/vip.h
SIGNATURES = {
    "vip_abi_version": (_c_int, []),
    "vip_launched_kernels": (_c_int, [ctypes.c_char_p, _c_size_t]),
    "vip_kernel_timing_begin": (_c_int, [_c_int]),
    "vip_kernel_timing_end": (_c_int, []),
    "vip_kernel_timing_get": (_c_int, [_c_int, ctypes.POINTER(_c_float), ctypes.c_char_p, _c_size_t]),
    "vip_error_string": (ctypes.c_char_p, [_c_int]),
    "vip_max_radius": (_c_int, []),
    "vip_max_ksize": (_c_int, [_c_int]),
    "vip_set_stencil_path": (_c_int, [_c_int]),
    "vip_texture_scratch_bytes": (_c_size_t, [_c_int, _c_int]),
    "vip_malloc": (_c_int, [ctypes.POINTER(_c_void_p), _c_size_t]),
    "vip_free": (_c_int, [_c_void_p]),
    "vip_upload": (_c_int, [_c_void_p, _c_void_p, _c_size_t]),
    "vip_download": (_c_int, [_c_void_p, _c_void_p, _c_size_t]),
    "vip_device_synchronize": (_c_int, []),
    "vip_device_count": (_c_int, [ctypes.POINTER(_c_int)]),
    "vip_set_device": (_c_int, [_c_int]),
    "vip_get_device": (_c_int, [ctypes.POINTER(_c_int)]),
    "vip_stream_synchronize": (_c_int, [_c_void_p]),
    "vip_host_alloc": (_c_int, [ctypes.POINTER(_c_void_p), _c_size_t]),
    "vip_host_free": (_c_int, [_c_void_p]),
    "vip_upload_async": (_c_int, [_c_void_p, _c_void_p, _c_size_t, _c_void_p]),
    "vip_download_async": (_c_int, [_c_void_p, _c_void_p, _c_size_t, _c_void_p]),
    "vip_stream_create": (_c_int, [ctypes.POINTER(_c_void_p)]),
    "vip_stream_destroy": (_c_int, [_c_void_p]),
    "vip_event_create": (_c_int, [ctypes.POINTER(_c_void_p)]),
    "vip_event_destroy": (_c_int, [_c_void_p]),
    "vip_event_record": (_c_int, [_c_void_p, _c_void_p]),
    "vip_stream_wait_event": (_c_int, [_c_void_p, _c_void_p]),
    "vip_event_synchronize": (_c_int, [_c_void_p]),
    "vip_bilateral_create": (_c_int, [ctypes.POINTER(_c_void_p), _c_int, _c_int, _c_int, _c_float, _c_float, _c_int]),
    "vip_bilateral_destroy": (_c_int, [_c_void_p]),
    "vip_bilateral_run": (_c_int, [_c_void_p, _c_void_p, _c_size_t, _c_void_p, _c_size_t, _c_void_p]),
    "vip_joint_bilateral_run": (
        _c_int, [_c_void_p, _c_void_p, _c_size_t, _c_void_p, _c_size_t, _c_void_p, _c_size_t, _c_void_p]),
    "vip_bilateral_run_rows": (
        _c_int, [_c_void_p, _c_void_p, _c_size_t, _c_void_p, _c_size_t, _c_void_p, _c_size_t,
                 _c_int, _c_int, _c_int, _c_int, _c_void_p]),
    "vip_bilateral_run_rows_batch": (
        _c_int, [_c_void_p, _c_int, ctypes.POINTER(_c_void_p), _c_size_t, ctypes.POINTER(_c_void_p), _c_size_t,
                 _c_int, _c_int, _c_int, _c_int, _c_int, _c_void_p]),
    "vip_adaptive_create": (_c_int, [ctypes.POINTER(_c_void_p), _c_int, _c_int, _c_int, _c_float, _c_float, _c_int]),
    "vip_adaptive_destroy": (_c_int, [_c_void_p]),
    "vip_adaptive_run": (_c_int, [_c_void_p, _c_void_p, _c_size_t, _c_void_p, _c_size_t, _c_void_p]),
    "vip_adaptive_run_rows": (
        _c_int, [_c_void_p, _c_void_p, _c_size_t, _c_void_p, _c_size_t, _c_int, _c_int, _c_int, _c_int, _c_void_p]),
    "vip_adaptive_run_rows_batch": (
        _c_int, [_c_void_p, _c_int, ctypes.POINTER(_c_void_p), _c_size_t, ctypes.POINTER(_c_void_p), _c_size_t,
                 _c_int, _c_int, _c_int, _c_int, _c_int, _c_void_p]),
    "vip_gradient_u8": (_c_int, [_c_void_p, _c_void_p, _c_int, _c_int, _c_int, _c_int, _c_void_p]),
    "vip_gradient_f32": (_c_int, [_c_void_p, _c_void_p, _c_int, _c_int, _c_int, _c_int, _c_void_p]),
    "vip_texture_create": (_c_int, [ctypes.POINTER(_c_void_p), _c_int, _c_int, _c_int, _c_int, _c_int]),
    "vip_texture_destroy": (_c_int, [_c_void_p]),
    "vip_texture_run": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "vip_texture_run_timed": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, ctypes.POINTER(_c_void_p)]),
    "vip_texture_halo_rows": (_c_int, [_c_int]),
    "vip_texture_set_mode": (_c_int, [_c_void_p, _c_int]),
    "vip_bilateral_set_waves": (_c_int, [_c_int]),
    "vip_bilateral_set_wide": (_c_int, [_c_int]),
    "vip_bilateral_set_frames_in_flight": (_c_int, [_c_int]),
    "vip_texture_iterate_rows": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_size_t, _c_int, _c_int, _c_int, _c_int,
                                          _c_void_p]),
    "vip_texture_blur_rtv": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "vip_texture_guide": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
}

_lock = threading.Lock()
_lib = None


class VipError(RuntimeError):
    """A non-zero status from the C ABI (hipError_t or VIP_ERR_*)."""

    def __init__(self, func: str, code: int):
        self.code = code
        msg = lib().vip_error_string(code).decode()
        super().__init__(f"{func} failed with status {code}: {msg}")


def lib() -> ctypes.CDLL:
    """Load libvip_hip.so (once). Raises if it is missing: there is no CPU path."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"{LIB_PATH} is not built; run __graft_entry__.build() "
                    "(make -C various_image_processings_amd/csrc)")
            handle = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
    return _lib


def check(func: str, code: int) -> None:
    if code != 0:
        raise VipError(func, code)


def call(name: str, *args) -> None:
    check(name, getattr(lib(), name)(*args))
