"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of oracle/liboracle.so (vip_oracle.c).

Parity status: pinned where the reference ships an executable oracle. The REF
profile equals the reference tests' own CPU oracles (test/adaptive_bilateral_filter.cu,
test/bilateral_texture_filter.cu, test/gradient.cu Ref* code, compiled in place by
oracle/Makefile) bit for bit on tests/golden/ref_oracles.npz: adaptive, gradient,
blur/mRTV and guide are pinned. Bilateral / joint bilateral stay "parity unpinned":
their only reference oracle is cv::bilateralFilter (OpenCV, absent here). The
mt19937 input generator is pinned to test/random_array.hpp (tests/golden).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use this.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
CUDA = 0  # src/<filter>_impl.cu numerics (float LUT coefficients, fma accumulate)
CPP = 1   # include/cpp numerics (double LUT coefficients, mul + add)
REF = 2   # the reference tests' own CPU oracles (test/*.cu Ref*: float LUT, mul + add, expf)

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i, f, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
        L.vipo_random_u8.argtypes = [sz, i, vp]
        L.vipo_random_f32.argtypes = [sz, f, vp]
        L.vipo_space_lut.argtypes = [i, f, i, vp]
        L.vipo_color_lut.argtypes = [i, f, i, vp]
        L.vipo_bilateral.argtypes = [vp, vp, vp, i, i, i, f, f, i]
        L.vipo_bilateral_rows.argtypes = [vp, vp, vp, i, i, i, f, f, i, i, i]
        L.vipo_adaptive.argtypes = [vp, vp, i, i, i, f, f, i]
        L.vipo_adaptive_rows.argtypes = [vp, vp, i, i, i, f, f, i, i, i]
        L.vipo_gradient_u8.argtypes = [vp, vp, i, i, i, i]
        L.vipo_gradient_f32.argtypes = [vp, vp, i, i, i, i]
        L.vipo_blur_rtv.argtypes = [vp, vp, vp, vp, i, i, i, i]
        L.vipo_guide.argtypes = [vp, vp, vp, i, i, i, i]
        L.vipo_texture.argtypes = [vp, vp, i, i, i, i, i]
        L.vipo_set_variant.argtypes = [i]
        for fn in ("vipo_random_u8", "vipo_random_f32", "vipo_space_lut", "vipo_color_lut", "vipo_bilateral",
                   "vipo_bilateral_rows", "vipo_adaptive", "vipo_adaptive_rows", "vipo_gradient_u8",
                   "vipo_gradient_f32", "vipo_blur_rtv", "vipo_guide", "vipo_texture", "vipo_set_variant"):
            getattr(L, fn).restype = None
        _lib = L
    return _lib


def _p(a: np.ndarray) -> int:
    assert a.flags.c_contiguous
    return a.ctypes.data


# ---- numerics-sensitivity variants of the CUDA profile (vip_oracle.c) ----
V_SUMK_FMA, V_BLEND_B, V_BLEND_NO, V_EXP_UP, V_EXP_DOWN = 1, 2, 4, 8, 16
VARIANTS = {"sumk_fma": V_SUMK_FMA, "blend_other_fma": V_BLEND_B, "blend_no_fma": V_BLEND_NO,
            "exp_plus_1ulp": V_EXP_UP, "exp_minus_1ulp": V_EXP_DOWN}


class variant:
    """Context manager: CUDA-profile calls inside use the given variant flags
    (process-global state of the oracle library; not thread-safe across variants)."""

    def __init__(self, flags: int):
        self.flags = flags

    def __enter__(self):
        lib().vipo_set_variant(self.flags)
        return self

    def __exit__(self, *exc):
        lib().vipo_set_variant(0)


# ---- inputs: test/random_array.hpp:9-31 ----
def random_u8(n: int, max_: int = 255) -> np.ndarray:
    out = np.empty(n, np.uint8)
    lib().vipo_random_u8(n, max_, _p(out))
    return out


def random_f32(n: int, max_: float = 255.0) -> np.ndarray:
    out = np.empty(n, np.float32)
    lib().vipo_random_f32(n, max_, _p(out))
    return out


def random_image(width: int, height: int) -> np.ndarray:
    """The reference tests' input: random_array<uint8_t>(w*h*3) viewed as HxWx3."""
    return random_u8(width * height * 3).reshape(height, width, 3)


def space_lut(ksize: int, sigma_space: float, profile: int = CUDA) -> np.ndarray:
    out = np.empty(ksize * ksize, np.float32)
    lib().vipo_space_lut(ksize, sigma_space, profile, _p(out))
    return out.reshape(ksize, ksize)


def color_lut(n: int, sigma_color: float, profile: int = CUDA) -> np.ndarray:
    out = np.empty(n, np.float32)
    lib().vipo_color_lut(n, sigma_color, profile, _p(out))
    return out


# ---- filters (HxWx3 uint8 in, HxWx3 uint8 out) ----
def _img(a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    assert a.ndim == 3 and a.shape[2] == 3
    return a


def bilateral(src, ksize=9, sigma_space=10.0, sigma_color=30.0, profile=CUDA, guide=None, threads=1):
    src = _img(src)
    g = None if guide is None else _img(guide)
    h, w, _ = src.shape
    dst = np.empty_like(src)
    L = lib()
    if threads <= 1:
        L.vipo_bilateral(_p(src), None if g is None else _p(g), _p(dst), w, h, ksize, sigma_space, sigma_color,
                         profile)
        return dst
    # row bands in parallel: ctypes releases the GIL for the C call
    bands = np.array_split(np.arange(h), threads)

    def run(rows):
        if len(rows) == 0:
            return
        r0 = int(rows[0])
        L.vipo_bilateral_rows(_p(src), None if g is None else _p(g), dst.ctypes.data + r0 * w * 3, w, h, ksize,
                              sigma_space, sigma_color, profile, r0, len(rows))

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(run, bands))
    return dst


def joint_bilateral(src, guide, ksize=9, sigma_space=10.0, sigma_color=30.0, profile=CUDA, threads=1):
    return bilateral(src, ksize, sigma_space, sigma_color, profile, guide=guide, threads=threads)


def bilateral_rows(src, row0, rows, ksize=9, sigma_space=10.0, sigma_color=30.0, profile=CUDA):
    src = _img(src)
    h, w, _ = src.shape
    dst = np.empty((rows, w, 3), np.uint8)
    lib().vipo_bilateral_rows(_p(src), None, _p(dst), w, h, ksize, sigma_space, sigma_color, profile, row0, rows)
    return dst


def joint_bilateral_rows(src, guide, row0, rows, ksize=9, sigma_space=10.0, sigma_color=30.0, profile=CUDA):
    src, guide = _img(src), _img(guide)
    h, w, _ = src.shape
    dst = np.empty((rows, w, 3), np.uint8)
    lib().vipo_bilateral_rows(_p(src), _p(guide), _p(dst), w, h, ksize, sigma_space, sigma_color, profile, row0, rows)
    return dst


def adaptive_rows(src, row0, rows, ksize=9, sigma_space=10.0, sigma_color=30.0, profile=CUDA):
    src = _img(src)
    h, w, _ = src.shape
    dst = np.empty((rows, w, 3), np.uint8)
    lib().vipo_adaptive_rows(_p(src), _p(dst), w, h, ksize, sigma_space, sigma_color, profile, row0, rows)
    return dst


def texture_rows(src, row0, rows, ksize=9, nitr=3, profile=CUDA):
    """Rows [row0, row0 + rows) of texture(src): the filter run on a crop with a
    ghost margin of nitr * (halo of one iteration) rows on each side (clipped at the
    frame edges, which are the crop's own edges there), so the band is exact."""
    src = _img(src)
    h = src.shape[0]
    m = nitr * ((ksize - 1) + 2 * (ksize // 2) + 1)
    a, b = max(0, row0 - m), min(h, row0 + rows + m)
    return texture(src[a:b], ksize, nitr, profile)[row0 - a:row0 - a + rows]


def bands(fn, spans, threads=8):
    """[fn(row0, rows) for (row0, rows) in spans], evaluated in parallel threads
    (the C calls release the GIL)."""
    with ThreadPoolExecutor(min(threads, len(spans))) as ex:
        return list(ex.map(lambda sp: fn(*sp), spans))


def adaptive(src, ksize=9, sigma_space=10.0, sigma_color=30.0, profile=CUDA, threads=1):
    src = _img(src)
    h, w, _ = src.shape
    dst = np.empty_like(src)
    L = lib()
    if threads <= 1:
        L.vipo_adaptive(_p(src), _p(dst), w, h, ksize, sigma_space, sigma_color, profile)
        return dst
    bands = np.array_split(np.arange(h), threads)

    def run(rows):
        if len(rows):
            r0 = int(rows[0])
            L.vipo_adaptive_rows(_p(src), dst.ctypes.data + r0 * w * 3, w, h, ksize, sigma_space, sigma_color,
                                 profile, r0, len(rows))

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(run, bands))
    return dst


def gradient(src, profile=CUDA):
    """src: HxW or HxWxC, uint8 or float32 -> HxW float32."""
    src = np.ascontiguousarray(src)
    h, w = src.shape[:2]
    ch = 1 if src.ndim == 2 else src.shape[2]
    dst = np.empty((h, w), np.float32)
    if src.dtype == np.uint8:
        lib().vipo_gradient_u8(_p(src), _p(dst), w, h, ch, profile)
    elif src.dtype == np.float32:
        lib().vipo_gradient_f32(_p(src), _p(dst), w, h, ch, profile)
    else:
        raise TypeError(src.dtype)
    return dst


def blur_rtv(image, magnitude, ksize, profile=CUDA):
    image = _img(image)
    magnitude = np.ascontiguousarray(magnitude, dtype=np.float32)
    h, w, _ = image.shape
    blurred = np.empty((h, w, 3), np.float32)
    rtv = np.empty((h, w), np.float32)
    lib().vipo_blur_rtv(_p(image), _p(magnitude), _p(blurred), _p(rtv), w, h, ksize, profile)
    return blurred, rtv


def guide(blurred, rtv, ksize, profile=CUDA):
    blurred = np.ascontiguousarray(blurred, dtype=np.float32)
    rtv = np.ascontiguousarray(rtv, dtype=np.float32)
    h, w = rtv.shape
    out = np.empty((h, w, 3), np.uint8)
    lib().vipo_guide(_p(blurred), _p(rtv), _p(out), w, h, ksize, profile)
    return out


def texture(src, ksize=9, nitr=3, profile=CUDA):
    src = _img(src)
    h, w, _ = src.shape
    dst = np.empty_like(src)
    lib().vipo_texture(_p(src), _p(dst), w, h, ksize, nitr, profile)
    return dst
