"""Python mirror of the reference's include/cuda/*.hpp API, over the C ABI.

Same class and method names, argument meaning and defaults as
yuyuyu-bot/various_image_processings:

* ``CudaBilateralFilter(width, height, ksize=9, sigma_space=10., sigma_color=30.)``
  with ``bilateral_filter(d_src, d_dst)`` and ``joint_bilateral_filter(d_src, d_guide, d_dst)``
  (include/cuda/bilateral_filter.hpp:9-24)
* ``CudaAdaptiveBilateralFilter(...).execute(d_src, d_dst)`` (adaptive_bilateral_filter.hpp:9-19)
* ``CudaBilateralTextureFilter(width, height, ksize=9, nitr=3).execute(d_src, d_dst)``
  (bilateral_texture_filter.hpp:9-12)
* ``cuda_gradient(d_src, d_dst, width, height, src_ch=1)`` (gradient.hpp:13-23)
* ``DeviceImage(width, height, channels=1, dtype)`` with upload/download/get (device_image.hpp:4-16)

Images are device buffers: a ``torch.Tensor`` on a HIP device (dense, uint8 for
images, float32 for magnitude/blurred/rtv) or a raw device address (int). Public
methods synchronise the device like the reference's; ``impl_`` exposes the
non-synchronising calls the reference's tests drive, plus an optional ``stream``.
Errors raise :class:`VipError` (the reference printed them and carried on).
"""
from __future__ import annotations

import ctypes
from typing import Optional

from . import _lib
from ._lib import VIP_NUMERICS_CPP, VIP_NUMERICS_CUDA, VipError, call, lib

__all__ = [
    "CudaBilateralFilter", "CudaAdaptiveBilateralFilter", "CudaBilateralTextureFilter", "cuda_gradient",
    "DeviceImage", "VipError", "VIP_NUMERICS_CUDA", "VIP_NUMERICS_CPP", "device_synchronize",
    "set_bilateral_waves", "set_bilateral_wide", "set_bilateral_frames_in_flight", "launched_kernels", "kernel_timing", "set_stencil_path", "max_ksize",
]


def _ptr(buf, nbytes: int = 0, dtype: str = "uint8") -> int:
    """Device address of a dense device buffer holding at least `nbytes` of `dtype`.

    Accepts a torch tensor on the current HIP device (checked: device, density,
    dtype, size -- a wrong-shaped tensor must raise here, not fault the GPU), a
    DeviceImage (size checked), or a raw int address (unchecked: the caller's
    responsibility, as in the reference's pointer API)."""
    if isinstance(buf, int):
        return buf
    if isinstance(buf, DeviceImage):
        if buf.dtype != dtype:
            raise ValueError(f"expected a {dtype} DeviceImage, got {buf.dtype}")
        if buf.nbytes < nbytes:
            raise ValueError(f"DeviceImage of {buf.nbytes} bytes, {nbytes} needed")
        return buf.get()
    if hasattr(buf, "data_ptr"):
        if not buf.is_cuda:
            raise ValueError("expected a device tensor (torch.cuda / HIP), got a host tensor")
        import torch
        if buf.device.index != torch.cuda.current_device():
            raise ValueError(f"tensor on {buf.device}, but the current device is cuda:{torch.cuda.current_device()}")
        if not buf.is_contiguous():
            raise ValueError("expected a dense (contiguous) tensor")
        want = {"uint8": torch.uint8, "float32": torch.float32}[dtype]
        if buf.dtype != want:
            raise ValueError(f"expected a {dtype} tensor, got {buf.dtype}")
        have = buf.numel() * buf.element_size()
        if have < nbytes:
            raise ValueError(f"tensor of {have} bytes, {nbytes} needed ({tuple(buf.shape)})")
        return buf.data_ptr()
    raise TypeError(f"cannot take a device pointer of {type(buf).__name__}")


def _stream(stream) -> Optional[int]:
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream  # torch.cuda.Stream


def device_synchronize() -> None:
    call("vip_device_synchronize")


def set_stencil_path(path: int = _lib.VIP_PATH_AUTO) -> None:
    """Process-wide kernel selection (include/vip.h vip_set_stencil_path; no reference
    counterpart): VIP_PATH_AUTO (radius-specialised kernels for radius 1..15, the
    runtime-radius kernel for 0 and 16..32) or VIP_PATH_RUNTIME (the runtime-radius
    kernel for every radius). Outputs are identical either way."""
    call("vip_set_stencil_path", int(path))


def max_ksize(filter_kind: int) -> int:
    """Largest ksize a filter accepts (include/vip.h vip_max_ksize): what the reference
    runs -- bilateral 65, joint 47, adaptive 63, texture 24."""
    return int(lib().vip_max_ksize(int(filter_kind)))


def set_bilateral_wide(mode: int = 0) -> None:
    """Companion tuning knob (include/vip.h vip_bilateral_set_wide): 0 = tile shape chosen
    per launch, 1 = 128-pixel tiles (8 outputs per thread), 2 = 256-pixel tiles (one row
    per wave, 4 outputs per thread). Outputs are identical for every setting."""
    call("vip_bilateral_set_wide", int(mode))


def set_bilateral_frames_in_flight(n: int = 0) -> None:
    """include/vip.h vip_bilateral_set_frames_in_flight: 0 = counted from the streams in use
    (default), 1..4 forced. A measurement knob; results are identical for every setting."""
    call("vip_bilateral_set_frames_in_flight", int(n))


def launched_kernels() -> list:
    """include/vip.h vip_launched_kernels: the kernels this thread launched through the
    library since the previous call, as the profiler names them (template arguments, no
    parameter list); clears the list."""
    n = lib().vip_launched_kernels(None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    lib().vip_launched_kernels(buf, n + 1)
    return [x for x in buf.value.decode().split("\n") if x]


class kernel_timing:
    """include/vip.h vip_kernel_timing_*: inside ``with kernel_timing(capacity) as kt:`` the
    next `capacity` kernels this thread launches through the library carry events the
    runtime stamps with each kernel's own begin and end (hipExtLaunchKernel). Afterwards
    ``kt.records()`` gives [(kernel name, ms)] in launch order and ``kt.durations()``
    {kernel name: [ms, ...]}; both wait for the kernels to finish."""

    def __init__(self, capacity: int):
        self.capacity = int(capacity)
        self.count = 0

    def __enter__(self):
        call("vip_kernel_timing_begin", self.capacity)
        return self

    def __exit__(self, *exc):
        self.count = int(lib().vip_kernel_timing_end())

    def records(self) -> list:
        out, ms, name = [], ctypes.c_float(), ctypes.create_string_buffer(512)
        for i in range(self.count):
            call("vip_kernel_timing_get", i, ctypes.byref(ms), name, len(name))
            out.append((name.value.decode(), float(ms.value)))
        return out

    def durations(self) -> dict:
        d = {}
        for n, ms in self.records():
            d.setdefault(n, []).append(ms)
        return d


def set_bilateral_waves(waves: int = 0) -> None:
    """Process-wide tuning knob (include/vip.h vip_bilateral_set_waves; no reference
    counterpart): waves per workgroup of the plain bilateral kernel for radius <= 8.
    0 = chosen per launch (small frames take smaller tiles), or 16 / 8 / 4. Outputs are
    identical for every setting."""
    call("vip_bilateral_set_waves", int(waves))


class _Handle:
    _destroy = ""

    def __init__(self):
        self._h = ctypes.c_void_p()

    def close(self) -> None:
        if self._h and self._h.value:
            getattr(lib(), self._destroy)(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _BilateralImpl(_Handle):
    """CudaBilateralFilter::Impl (src/bilateral_filter_impl.cuh:7-33): no synchronisation."""
    _destroy = "vip_bilateral_destroy"

    def __init__(self, width, height, ksize=9, sigma_space=10.0, sigma_color=30.0, numerics=VIP_NUMERICS_CUDA):
        super().__init__()
        self.width, self.height, self.ksize = int(width), int(height), int(ksize)
        call("vip_bilateral_create", ctypes.byref(self._h), self.width, self.height, self.ksize,
             float(sigma_space), float(sigma_color), int(numerics))

    def bilateral_filter(self, d_src, d_dst, stream=None):
        p, n = self.width * 3, self.width * 3 * self.height
        call("vip_bilateral_run", self._h, _ptr(d_src, n), p, _ptr(d_dst, n), p, _stream(stream))

    def joint_bilateral_filter(self, d_src, d_guide, d_dst, stream=None):
        p, n = self.width * 3, self.width * 3 * self.height
        call("vip_joint_bilateral_run", self._h, _ptr(d_src, n), p, _ptr(d_guide, n), p, _ptr(d_dst, n), p,
             _stream(stream))

    def run_rows(self, d_src, d_dst, out_rows, src_row0, row_lo, row_hi, d_guide=None, stream=None):
        """Row-band filter for row-sharded frames (include/vip.h vip_bilateral_run_rows):
        d_src (and d_guide) hold rows [0, row_hi) at least, d_dst out_rows rows."""
        p = self.width * 3
        g = None if d_guide is None else _ptr(d_guide, p * int(row_hi))
        call("vip_bilateral_run_rows", self._h, _ptr(d_src, p * int(row_hi)), p, g, p, _ptr(d_dst, p * int(out_rows)),
             p, int(out_rows), int(src_row0), int(row_lo), int(row_hi), _stream(stream))

    def run_rows_batch(self, d_srcs, d_dsts, out_rows, src_row0, row_lo, row_hi, free_cus=0, stream=None):
        """run_rows over several frames of the same geometry, up to 6 per launch
        (include/vip.h vip_bilateral_run_rows_batch)."""
        _run_batch("vip_bilateral_run_rows_batch", self._h, self.width * 3, d_srcs, d_dsts, out_rows, src_row0,
                   row_lo, row_hi, free_cus, stream)


def _run_batch(name, h, p, d_srcs, d_dsts, out_rows, src_row0, row_lo, row_hi, free_cus, stream):
    if len(d_srcs) != len(d_dsts):
        raise ValueError("one output per input frame")
    n = len(d_srcs)
    srcs = (ctypes.c_void_p * max(n, 1))(*[_ptr(x, p * int(row_hi)) for x in d_srcs])
    dsts = (ctypes.c_void_p * max(n, 1))(*[_ptr(x, p * int(out_rows)) for x in d_dsts])
    call(name, h, n, srcs, p, dsts, p, int(out_rows), int(src_row0), int(row_lo), int(row_hi), int(free_cus),
         _stream(stream))


class CudaBilateralFilter:
    """include/cuda/bilateral_filter.hpp:7-29; public calls block until done (:299, :309)."""

    def __init__(self, width, height, ksize=9, sigma_space=10.0, sigma_color=30.0, numerics=VIP_NUMERICS_CUDA):
        self.impl_ = _BilateralImpl(width, height, ksize, sigma_space, sigma_color, numerics)

    def bilateral_filter(self, d_src, d_dst):
        self.impl_.bilateral_filter(d_src, d_dst)
        device_synchronize()

    def joint_bilateral_filter(self, d_src, d_guide, d_dst):
        self.impl_.joint_bilateral_filter(d_src, d_guide, d_dst)
        device_synchronize()


class _AdaptiveImpl(_Handle):
    """CudaAdaptiveBilateralFilter::Impl (src/adaptive_bilateral_filter_impl.cuh:7-29)."""
    _destroy = "vip_adaptive_destroy"

    def __init__(self, width, height, ksize=9, sigma_space=10.0, sigma_color=30.0, numerics=VIP_NUMERICS_CUDA):
        super().__init__()
        self.width, self.height, self.ksize = int(width), int(height), int(ksize)
        call("vip_adaptive_create", ctypes.byref(self._h), self.width, self.height, self.ksize,
             float(sigma_space), float(sigma_color), int(numerics))

    def execute(self, d_src, d_dst, stream=None):
        p, n = self.width * 3, self.width * 3 * self.height
        call("vip_adaptive_run", self._h, _ptr(d_src, n), p, _ptr(d_dst, n), p, _stream(stream))

    def run_rows(self, d_src, d_dst, out_rows, src_row0, row_lo, row_hi, stream=None):
        p = self.width * 3
        call("vip_adaptive_run_rows", self._h, _ptr(d_src, p * int(row_hi)), p, _ptr(d_dst, p * int(out_rows)), p,
             int(out_rows), int(src_row0), int(row_lo), int(row_hi), _stream(stream))

    def run_rows_batch(self, d_srcs, d_dsts, out_rows, src_row0, row_lo, row_hi, free_cus=0, stream=None):
        """include/vip.h vip_adaptive_run_rows_batch"""
        _run_batch("vip_adaptive_run_rows_batch", self._h, self.width * 3, d_srcs, d_dsts, out_rows, src_row0,
                   row_lo, row_hi, free_cus, stream)


class CudaAdaptiveBilateralFilter:
    """include/cuda/adaptive_bilateral_filter.hpp:7-24."""

    def __init__(self, width, height, ksize=9, sigma_space=10.0, sigma_color=30.0, numerics=VIP_NUMERICS_CUDA):
        self.impl_ = _AdaptiveImpl(width, height, ksize, sigma_space, sigma_color, numerics)

    def execute(self, d_src, d_dst):
        self.impl_.execute(d_src, d_dst)
        device_synchronize()


class _TextureImpl(_Handle):
    """CudaBilateralTextureFilter::Impl (src/bilateral_texture_filter_impl.cuh:7-45)."""
    _destroy = "vip_texture_destroy"

    def __init__(self, width, height, ksize=9, nitr=3, numerics=VIP_NUMERICS_CUDA):
        super().__init__()
        self.width, self.height, self.ksize, self.nitr = int(width), int(height), int(ksize), int(nitr)
        call("vip_texture_create", ctypes.byref(self._h), self.width, self.height, self.ksize, self.nitr,
             int(numerics))

    TWO_LAUNCH, FUSED = 0, 1  # include/vip.h VIP_TEXTURE_*

    def set_mode(self, mode):
        """TWO_LAUNCH (default) or FUSED (ksize 5: guide + JBF in one launch per
        iteration, the guide kept in LDS); include/vip.h vip_texture_set_mode."""
        call("vip_texture_set_mode", self._h, int(mode))

    def execute(self, d_src, d_dst, stream=None):
        n = self.width * self.height * 3
        call("vip_texture_run", self._h, _ptr(d_src, n), _ptr(d_dst, n), _stream(stream))

    def execute_timed(self, d_src, d_dst, events, stream=None):
        """execute() with per-stage timestamps (include/vip.h vip_texture_run_timed):
        `events` = 2 * nitr + 1 torch.cuda.Event(enable_timing=True), recorded before
        each iteration's guide stage, before its joint bilateral, and after the last."""
        n = self.width * self.height * 3
        if len(events) != 2 * self.nitr + 1:
            raise ValueError(f"need {2 * self.nitr + 1} events, got {len(events)}")
        for e in events:  # torch creates the HIP event lazily, at its first record
            if not e.cuda_event:
                e.record(stream) if stream is not None and not isinstance(stream, int) else e.record()
        arr = (ctypes.c_void_p * len(events))(*[e.cuda_event for e in events])
        call("vip_texture_run_timed", self._h, _ptr(d_src, n), _ptr(d_dst, n), _stream(stream), arr)

    def compute_blur_and_rtv(self, d_image, d_magnitude, d_blurred, d_rtv, stream=None):
        n = self.width * self.height
        call("vip_texture_blur_rtv", self._h, _ptr(d_image, 3 * n), _ptr(d_magnitude, 4 * n, "float32"),
             _ptr(d_blurred, 12 * n, "float32"), _ptr(d_rtv, 4 * n, "float32"), _stream(stream))

    def compute_guide(self, d_blurred, d_rtv, d_guide, stream=None):
        n = self.width * self.height
        call("vip_texture_guide", self._h, _ptr(d_blurred, 12 * n, "float32"), _ptr(d_rtv, 4 * n, "float32"),
             _ptr(d_guide, 3 * n), _stream(stream))

    def iterate_rows(self, d_src, d_dst, out_row0, out_rows, row_lo, row_hi, stream=None):
        """One iteration on a row slab (include/vip.h vip_texture_iterate_rows): d_dst
        receives slab rows [out_row0, out_row0 + out_rows)."""
        p = self.width * 3
        call("vip_texture_iterate_rows", self._h, _ptr(d_src, p * self.height), _ptr(d_dst, p * int(out_rows)), p,
             int(out_row0), int(out_rows), int(row_lo), int(row_hi), _stream(stream))


class CudaBilateralTextureFilter:
    """include/cuda/bilateral_texture_filter.hpp:7-17."""

    def __init__(self, width, height, ksize=9, nitr=3, numerics=VIP_NUMERICS_CUDA):
        self.impl_ = _TextureImpl(width, height, ksize, nitr, numerics)

    def execute(self, d_src, d_dst):
        self.impl_.execute(d_src, d_dst)
        device_synchronize()


def cuda_gradient(d_src, d_dst, width, height, src_ch=1, numerics=VIP_NUMERICS_CUDA, stream=None):
    """include/cuda/gradient.hpp:13-23. The source dtype (uint8 / float32, the
    reference's template argument T) is taken from a torch tensor or a DeviceImage; raw
    addresses are treated as uint8. Asynchronous, like src/gradient_impl.cu:90-103."""
    if isinstance(d_src, DeviceImage):
        is_f32 = d_src.dtype == "float32"
    else:
        is_f32 = hasattr(d_src, "dtype") and str(d_src.dtype) == "torch.float32"
    name = "vip_gradient_f32" if is_f32 else "vip_gradient_u8"
    n = int(width) * int(height)
    call(name, _ptr(d_src, n * int(src_ch) * (4 if is_f32 else 1), "float32" if is_f32 else "uint8"),
         _ptr(d_dst, 4 * n, "float32"), int(width), int(height), int(src_ch), int(numerics), _stream(stream))


class DeviceImage:
    """include/cuda/device_image.hpp:4-16: dense device buffer, blocking upload/download.
    ``dtype`` is 'uint8' or 'float32'; host data are numpy arrays (or buffer objects)."""

    _ITEM = {"uint8": 1, "float32": 4}

    def __init__(self, width, height, channels=1, dtype="uint8"):
        self.dtype = str(dtype)  # the reference's template argument T
        self.nbytes = int(width) * int(height) * int(channels) * self._ITEM[self.dtype]
        self._p = ctypes.c_void_p()
        call("vip_malloc", ctypes.byref(self._p), self.nbytes)

    def get(self) -> int:
        return self._p.value

    def upload(self, data) -> None:
        import numpy as np
        a = np.ascontiguousarray(data)
        if a.nbytes != self.nbytes:
            raise ValueError(f"upload of {a.nbytes} bytes into a {self.nbytes}-byte image")
        call("vip_upload", self._p, a.ctypes.data, self.nbytes)

    def download(self, out) -> None:
        import numpy as np
        if not (isinstance(out, np.ndarray) and out.flags.c_contiguous and out.nbytes == self.nbytes):
            raise ValueError("download target must be a dense numpy array of the image's size")
        call("vip_download", out.ctypes.data, self._p, self.nbytes)

    def __del__(self):
        try:
            if self._p and self._p.value:
                lib().vip_free(self._p)
                self._p = ctypes.c_void_p()
        except Exception:
            pass
