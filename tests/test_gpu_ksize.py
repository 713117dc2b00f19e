"""GPU parity at every ksize the reference runs.

The reference sizes its dynamic shared memory from ksize with no cap
(src/bilateral_filter_impl.cu:252-254, 272-275; src/adaptive_bilateral_filter_impl.cu:
165-167), so under CUDA's 48 KB default it filters with bilateral ksize up to 65, joint
up to 47, adaptive up to 63, texture k up to 24 (its JBF is 2k-1), and ksize 1
(radius 0). Radius 0 and 16..32 run on the runtime-radius kernel
(csrc/vip_stencil_rt.hip); the texture guide stage is specialised up to radius 12.

Bar: bit-exact against the oracle of the same numerics profile, on ragged frames and
on one full-width 3840-pixel band per filter that crosses the top border.
"""
import numpy as np
import pytest

import various_image_processings_amd as vip
from various_image_processings_amd.filters import _AdaptiveImpl, _BilateralImpl, _TextureImpl

pytestmark = pytest.mark.gpu

PROFILES = [(vip.VIP_NUMERICS_CUDA, 0), (vip.VIP_NUMERICS_CPP, 1)]


def _mismatch(a, b):
    d = np.argwhere(a != b)
    return f"{len(d)} mismatches, first {d[:5].tolist()}"


def _run_bilateral(dev, img, k, numerics=0, guide=None, ss=10.0, sc=30.0):
    h, w, _ = img.shape
    f = vip.CudaBilateralFilter(w, h, k, ss, sc, numerics=numerics)
    d_dst = dev.empty((h, w, 3))
    if guide is None:
        f.bilateral_filter(dev.put(img), d_dst)
    else:
        f.joint_bilateral_filter(dev.put(img), dev.put(guide), d_dst)
    return dev.get(d_dst)


def _run_adaptive(dev, img, k, numerics=0):
    h, w, _ = img.shape
    d_dst = dev.empty((h, w, 3))
    vip.CudaAdaptiveBilateralFilter(w, h, k, numerics=numerics).execute(dev.put(img), d_dst)
    return dev.get(d_dst)


def _run_texture(dev, img, k, nitr, numerics=0):
    h, w, _ = img.shape
    d_dst = dev.empty((h, w, 3))
    vip.CudaBilateralTextureFilter(w, h, k, nitr, numerics=numerics).execute(dev.put(img), d_dst)
    return dev.get(d_dst)


def _img(oracle, h, w, seed_rev=False):
    a = oracle.random_u8(h * w * 3).reshape(h, w, 3)
    return a[::-1, ::-1].copy() if seed_rev else a


RAGGED = [(1, 1), (37, 53), (70, 131), (130, 67)]


@pytest.mark.parametrize("k", [1, 33, 47, 65])
@pytest.mark.parametrize("shape", RAGGED)
@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_bilateral_large_and_unit_ksize(dev, oracle, k, shape, numerics, profile):
    img = _img(oracle, *shape)
    got = _run_bilateral(dev, img, k, numerics)
    want = oracle.bilateral(img, k, profile=profile)
    assert np.array_equal(got, want), _mismatch(got, want)
    if k == 1:  # radius 0: the centre tap alone, weight 1
        assert np.array_equal(got, img)


@pytest.mark.parametrize("k", [1, 33, 47])
@pytest.mark.parametrize("shape", RAGGED)
@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_joint_large_and_unit_ksize(dev, oracle, k, shape, numerics, profile):
    img = _img(oracle, *shape)
    guide = _img(oracle, *shape, seed_rev=True)
    got = _run_bilateral(dev, img, k, numerics, guide=guide)
    want = oracle.joint_bilateral(img, guide, k, profile=profile)
    assert np.array_equal(got, want), _mismatch(got, want)


@pytest.mark.parametrize("k", [1, 33, 63])
@pytest.mark.parametrize("shape", RAGGED)
@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_adaptive_large_and_unit_ksize(dev, oracle, k, shape, numerics, profile):
    img = _img(oracle, *shape)
    got = _run_adaptive(dev, img, k, numerics)
    want = oracle.adaptive(img, k, profile=profile)
    assert np.array_equal(got, want), _mismatch(got, want)


@pytest.mark.parametrize("k,nitr", [(1, 2), (17, 2), (18, 1), (24, 2)])
@pytest.mark.parametrize("shape", [(1, 1), (37, 53), (70, 131)])
@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_texture_large_and_unit_ksize(dev, oracle, k, nitr, shape, numerics, profile):
    img = _img(oracle, *shape)
    got = _run_texture(dev, img, k, nitr, numerics)
    want = oracle.texture(img, k, nitr, profile)
    assert np.array_equal(got, want), _mismatch(got, want)


@pytest.mark.parametrize("k", [7, 9, 11, 13, 15])
@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_texture_guide_tiles_across_tile_seams(dev, oracle, k, numerics, profile):
    """Texture ksize 7-15, the per-radius guide-stage tiles (vip_texture.hip GfTile: 92 x 32
    at R = 3-5, 64 x 16 at R = 6, 60 x 36 with capped VGPRs at R = 7), on a frame several
    tiles wide and tall with partial tiles on the right and bottom edges."""
    img = _img(oracle, 157, 263, seed_rev=True)
    got = _run_texture(dev, img, k, 2, numerics)
    want = oracle.texture(img, k, 2, profile)
    assert np.array_equal(got, want), _mismatch(got, want)


# One full-width 3840-pixel band per filter at its largest ksize: a 3840 x 200 frame
# (rows 0..199 with the replicate border on top), checked on rows crossing the top
# border and an interior tile seam.
BAND_W, BAND_H = 3840, 200


@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_bilateral_65_band(dev, oracle, numerics, profile):
    img = oracle.random_image(BAND_W, BAND_H)
    got = _run_bilateral(dev, img, 65, numerics)
    for r0 in (0, 60):
        want = oracle.bilateral_rows(img, r0, 6, 65, profile=profile)
        assert np.array_equal(got[r0:r0 + 6], want), (r0, _mismatch(got[r0:r0 + 6], want))


@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_joint_47_band(dev, oracle, numerics, profile):
    img = oracle.random_image(BAND_W, BAND_H)
    guide = img[::-1].copy()
    got = _run_bilateral(dev, img, 47, numerics, guide=guide)
    for r0 in (0, 60):
        want = oracle.joint_bilateral_rows(img, guide, r0, 6, 47, profile=profile)
        assert np.array_equal(got[r0:r0 + 6], want), (r0, _mismatch(got[r0:r0 + 6], want))


@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_adaptive_63_band(dev, oracle, numerics, profile):
    img = oracle.random_image(BAND_W, BAND_H)
    got = _run_adaptive(dev, img, 63, numerics)
    for r0 in (0, 60):
        want = oracle.adaptive_rows(img, r0, 6, 63, profile=profile)
        assert np.array_equal(got[r0:r0 + 6], want), (r0, _mismatch(got[r0:r0 + 6], want))


@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_texture_24_band(dev, oracle, numerics, profile):
    img = oracle.random_image(BAND_W, BAND_H)
    got = _run_texture(dev, img, 24, 1, numerics)
    for r0 in (0, 60):
        want = oracle.texture_rows(img, r0, 4, 24, 1, profile=profile)
        assert np.array_equal(got[r0:r0 + 4], want), (r0, _mismatch(got[r0:r0 + 4], want))


# The runtime-radius kernel at the templated radii: forced for every radius, it must give
# the templated kernels' (== the oracle's) bytes -- a check of its indexing at many radii.
@pytest.mark.parametrize("k", [3, 9, 15, 31])
def test_runtime_kernel_matches_templated(dev, oracle, k):
    img = _img(oracle, 70, 131)
    guide = _img(oracle, 70, 131, seed_rev=True)
    try:
        vip.set_stencil_path(vip.VIP_PATH_RUNTIME)
        got_b = _run_bilateral(dev, img, k)
        got_j = _run_bilateral(dev, img, k, guide=guide)
        got_a = _run_adaptive(dev, img, k, numerics=1)
    finally:
        vip.set_stencil_path(vip.VIP_PATH_AUTO)
    assert np.array_equal(got_b, _run_bilateral(dev, img, k))
    assert np.array_equal(got_j, _run_bilateral(dev, img, k, guide=guide))
    assert np.array_equal(got_a, _run_adaptive(dev, img, k, numerics=1))
    assert np.array_equal(got_b, oracle.bilateral(img, k))


def test_runtime_kernel_row_bands(dev, oracle):
    """vip_bilateral_run_rows / vip_adaptive_run_rows (the sharded path) at radius 20."""
    from various_image_processings_amd._lib import call
    img = oracle.random_image(150, 90)
    d_src = dev.put(img)
    for cls, fn in ((_BilateralImpl, oracle.bilateral), (_AdaptiveImpl, oracle.adaptive)):
        impl = cls(150, 90, 41)
        d_dst = dev.empty((30, 150, 3))
        # output rows 40..69, neighbours clamped to rows 25..84 of the frame
        if cls is _BilateralImpl:
            call("vip_bilateral_run_rows", impl._h, d_src.data_ptr(), 450, None, 0, d_dst.data_ptr(), 450, 30, 40,
                 25, 85, None)
        else:
            call("vip_adaptive_run_rows", impl._h, d_src.data_ptr(), 450, d_dst.data_ptr(), 450, 30, 40, 25, 85,
                 None)
        want = fn(img[25:85].copy(), 41)[15:45]
        got = dev.get(d_dst)
        assert np.array_equal(got, want), (cls.__name__, _mismatch(got, want))


def test_only_unsupported_ksizes_rejected(dev):
    """Even ksize (the reference's tile is sized for ksize - 1 apron columns but reads
    2 * (ksize / 2): undefined), ksize <= 0 and ksizes above what the reference runs are
    rejected; every other ksize builds a handle."""
    for k in range(-1, 70):
        ok_b = k >= 1 and k % 2 == 1 and k <= 65
        ok_a = k >= 1 and k % 2 == 1 and k <= 63
        ok_t = 1 <= k <= 24
        for cls, ok in ((_BilateralImpl, ok_b), (_AdaptiveImpl, ok_a)):
            if ok:
                cls(8, 8, k)
            else:
                with pytest.raises(vip.VipError) as e:
                    cls(8, 8, k)
                assert e.value.code == 10002, (cls.__name__, k)
        if ok_t:
            _TextureImpl(8, 8, k, 1)
        else:
            with pytest.raises(vip.VipError) as e:
                _TextureImpl(8, 8, k, 1)
            assert e.value.code == 10002, ("texture", k)
    # a bilateral handle above the joint limit filters, but its joint call is rejected
    # (the reference's launch fails on shared memory there and prints the error)
    f = vip.CudaBilateralFilter(8, 8, 49)
    d = dev.empty((8, 8, 3))
    f.bilateral_filter(dev.put(np.zeros((8, 8, 3), np.uint8)), d)
    with pytest.raises(vip.VipError) as e:
        f.joint_bilateral_filter(dev.put(np.zeros((8, 8, 3), np.uint8)), dev.put(np.zeros((8, 8, 3), np.uint8)), d)
    assert e.value.code == 10002


def test_texture_handle_allocates_no_f32_scratch(dev):
    """A 4K texture handle holds three u8x3 frames (75 MB), not the reference Impl's
    f32 magnitude / blurred / rtv buffers on top (241 MB)."""
    import torch
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    t = _TextureImpl(3840, 2160, 5, 5)
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    used = free0 - free1
    want = vip.lib().vip_texture_scratch_bytes(3840, 2160)
    assert want == 3 * 3840 * 2160 * 3
    # + the embedded JBF handle's LUT and tables (< 1 MiB) and allocator granularity
    assert want <= used <= want + 8 * 2 ** 20, (used, want)
    del t


@pytest.mark.parametrize("k", list(range(2, 25, 2)))
def test_texture_every_even_k_follows_include_cpp(dev, oracle, k):
    """Even texture ksize: the include/cpp semantics (a (k+1)x(k+1) window, the box sum
    over k*k, sigma_alpha 1/(5k); include/cpp/bilateral_texture_filter.hpp:41-59), which
    the oracle restates (tests/test_oracle.py::test_numpy_restatement_blur_rtv_guide); the
    reference's CUDA stages read one column past their tile there (undefined)."""
    img = _img(oracle, 41, 67)
    got = _run_texture(dev, img, k, 2)
    want = oracle.texture(img, k, 2)
    assert np.array_equal(got, want), _mismatch(got, want)
