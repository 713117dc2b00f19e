"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of oracle/_ref/libref_test_oracles.so, the
reference tests' own CPU oracles compiled where they lie (oracle/ref_test_oracles.cpp,
oracle/Makefile). Exists only in the dev container, where /root/reference is mounted:
tests/golden/make_ref_golden.py turns its outputs into the committed fixture
tests/golden/ref_oracles.npz, and tests/test_ref_pinned.py re-derives that fixture live
when the library is present. Nothing on the GPU box loads it."""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_ref", "libref_test_oracles.so")
_lib = None


def available() -> bool:
    return os.path.exists(LIB_PATH)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        L = ctypes.CDLL(LIB_PATH)
        vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.ref_adaptive.argtypes = [vp, vp, i, i, i, f, f]
        L.ref_blur_rtv.argtypes = [vp, vp, vp, vp, i, i, i]
        L.ref_guide.argtypes = [vp, vp, vp, i, i, i]
        L.ref_gradient_u8.argtypes = [vp, vp, i, i, i]
        L.ref_gradient_f32.argtypes = [vp, vp, i, i, i]
        L.ref_cpp_luts.argtypes = [i, f, f, i, vp, vp]
        for fn in ("ref_adaptive", "ref_blur_rtv", "ref_guide", "ref_gradient_u8", "ref_gradient_f32", "ref_cpp_luts"):
            getattr(L, fn).restype = None
        _lib = L
    return _lib


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def adaptive(src, ksize=9, sigma_space=10.0, sigma_color=30.0):
    """RefAdaptiveBilateralFilterImpl::execute (test/adaptive_bilateral_filter.cu:55-107)."""
    src = _c(src, np.uint8)
    h, w, _ = src.shape
    dst = np.empty_like(src)
    lib().ref_adaptive(src.ctypes.data, dst.ctypes.data, w, h, ksize, sigma_space, sigma_color)
    return dst


def blur_rtv(image, magnitude, ksize):
    """RefBilateralTextureFilterImpl::compute_blur_and_rtv (test/bilateral_texture_filter.cu:13-59)."""
    image, magnitude = _c(image, np.uint8), _c(magnitude, np.float32)
    h, w, _ = image.shape
    blurred = np.empty((h, w, 3), np.float32)
    rtv = np.empty((h, w), np.float32)
    lib().ref_blur_rtv(image.ctypes.data, magnitude.ctypes.data, blurred.ctypes.data, rtv.ctypes.data, w, h, ksize)
    return blurred, rtv


def guide(blurred, rtv, ksize):
    """RefBilateralTextureFilterImpl::compute_guide (test/bilateral_texture_filter.cu:61-104)."""
    blurred, rtv = _c(blurred, np.float32), _c(rtv, np.float32)
    h, w = rtv.shape
    out = np.empty((h, w, 3), np.uint8)
    lib().ref_guide(blurred.ctypes.data, rtv.ctypes.data, out.ctypes.data, w, h, ksize)
    return out


def gradient(src):
    """ref_gradient<T> (test/gradient.cu:9-34); src HxW or HxWxC, uint8 or float32."""
    src = np.ascontiguousarray(src)
    h, w = src.shape[:2]
    ch = 1 if src.ndim == 2 else src.shape[2]
    dst = np.empty((h, w), np.float32)
    fn = lib().ref_gradient_u8 if src.dtype == np.uint8 else lib().ref_gradient_f32
    fn(src.ctypes.data, dst.ctypes.data, w, h, ch)
    return dst


def cpp_luts(ksize, sigma_space, sigma_color, color_len=768):
    """internal::pre_compute_kernels (include/cpp/bilateral_filter.hpp:10-39): the include/cpp
    filters' space LUT (ksize x ksize) and colour LUT (768, or 1536 for the adaptive filter)."""
    space = np.empty((ksize, ksize), np.float32)
    color = np.empty(color_len, np.float32)
    lib().ref_cpp_luts(ksize, sigma_space, sigma_color, color_len, space.ctypes.data, color.ctypes.data)
    return space, color
