"""GPU parity tests: the HIP kernels (through the C ABI) against the CPU oracle.

Bar: bit-exact. The oracle's CUDA profile restates src/<filter>_impl.cu (float LUT
coefficients, fused multiply-add), its CPP profile include/cpp (double LUT
coefficients, multiply then add); the library implements both (numerics flag),
so every u8 output must match exactly, and f32 stage outputs bit for bit.
The reference's own tolerance (+-1 per channel, test/bilateral_filter.cu:58-60)
is asserted separately between profiles.
"""
import numpy as np
import pytest

import various_image_processings_amd as vip
from various_image_processings_amd.filters import _AdaptiveImpl, _BilateralImpl, _TextureImpl

pytestmark = pytest.mark.gpu

PROFILES = [(vip.VIP_NUMERICS_CUDA, 0), (vip.VIP_NUMERICS_CPP, 1)]


def _bilateral_gpu(dev, img, k, ss=10.0, sc=30.0, numerics=0, guide=None):
    h, w, _ = img.shape
    f = vip.CudaBilateralFilter(w, h, k, ss, sc, numerics=numerics)
    d_src, d_dst = dev.put(img), dev.empty((h, w, 3))
    if guide is None:
        f.bilateral_filter(d_src, d_dst)
    else:
        f.joint_bilateral_filter(d_src, dev.put(guide), d_dst)
    return dev.get(d_dst)


def _mismatch(a, b):
    d = np.argwhere(a != b)
    return f"{len(d)} mismatches, first {d[:5].tolist()} got {a[tuple(d[0])] if len(d) else None} " \
           f"want {b[tuple(d[0])] if len(d) else None}"


@pytest.mark.parametrize("k", [3, 5, 9, 11, 15, 21, 31])
@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_bilateral_reference_inputs(dev, oracle, k, numerics, profile):
    img = oracle.random_image(50, 50)
    got = _bilateral_gpu(dev, img, k, numerics=numerics)
    want = oracle.bilateral(img, k, profile=profile)
    assert np.array_equal(got, want), _mismatch(got, want)


@pytest.mark.parametrize("shape", [(1, 1), (2, 3), (5, 7), (33, 130), (70, 129), (64, 257), (17, 4), (129, 1)])
@pytest.mark.parametrize("k", [3, 15])
def test_bilateral_ragged_shapes(dev, oracle, shape, k):
    h, w = shape
    img = oracle.random_u8(h * w * 3).reshape(h, w, 3)
    got = _bilateral_gpu(dev, img, k)
    want = oracle.bilateral(img, k)
    assert np.array_equal(got, want), _mismatch(got, want)


@pytest.mark.parametrize("k,ss,sc", [(9, 10.0, 30.0), (15, 10.0, 30.0), (9, 4.0, 1.73205080757), (31, 20.0, 60.0)])
def test_bilateral_large_frame(dev, oracle, k, ss, sc):
    img = oracle.random_image(640, 360)
    got = _bilateral_gpu(dev, img, k, ss, sc)
    want = oracle.bilateral(img, k, ss, sc, threads=16)
    assert np.array_equal(got, want), _mismatch(got, want)


# Small frames run the plain kernel on 8 or 4 waves with 128x32 / 128x16 tiles
# (vip_bilateral_set_waves, radius <= 8). Every forced wave count must give the oracle's
# bytes; 1300x400 has 275 tiles at 4 waves, so some workgroups take two.
@pytest.mark.parametrize("waves", [16, 8, 4])
@pytest.mark.parametrize("wide", [1, 2])
@pytest.mark.parametrize("k", [3, 11, 17])
def test_bilateral_forced_waves(dev, oracle, waves, wide, k):
    """wide = 2: 256-pixel tiles, one row per wave, 4 outputs per thread (vip_bilateral_set_wide)."""
    img = oracle.random_image(1300, 400)
    vip.set_bilateral_waves(waves)
    vip.set_bilateral_wide(wide)
    try:
        got = _bilateral_gpu(dev, img, k)
    finally:
        vip.set_bilateral_waves(0)
        vip.set_bilateral_wide(0)
    want = oracle.bilateral(img, k, threads=16)
    assert np.array_equal(got, want), _mismatch(got, want)


@pytest.mark.parametrize("shape", [(1, 1), (7, 3840), (270, 3840), (17, 300), (512, 512), (33, 257)])
@pytest.mark.parametrize("k", [5, 15])
@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_bilateral_wide_tiles_auto(dev, oracle, shape, k, numerics, profile):
    """Frames the per-launch choice gives 256-pixel tiles (a 7-row edge band, the 270-row
    slab of the 4K frame at 8 GPUs, lenna 512^2), ragged widths, both profiles."""
    h, w = shape
    img = oracle.random_u8(h * w * 3).reshape(h, w, 3)
    got = _bilateral_gpu(dev, img, k, numerics=numerics)
    want = oracle.bilateral(img, k, profile=profile, threads=16)
    assert np.array_equal(got, want), _mismatch(got, want)


def test_bilateral_set_waves_rejects_other_counts():
    with pytest.raises(vip.VipError):
        vip.set_bilateral_waves(12)
    vip.set_bilateral_waves(0)
    with pytest.raises(vip.VipError):
        vip.set_bilateral_wide(3)
    vip.set_bilateral_wide(0)


@pytest.mark.parametrize("k", [3, 9, 15, 25, 31])
@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_joint_bilateral(dev, oracle, k, numerics, profile):
    img = oracle.random_image(70, 45)
    guide = oracle.random_u8(70 * 45 * 3)[::-1].copy().reshape(45, 70, 3)
    got = _bilateral_gpu(dev, img, k, numerics=numerics, guide=guide)
    want = oracle.joint_bilateral(img, guide, k, profile=profile)
    assert np.array_equal(got, want), _mismatch(got, want)


@pytest.mark.parametrize("k", [9, 25])
def test_joint_bilateral_multi_tile(dev, oracle, k):
    # 3000 x 700: 24 x 11 = 264 (P=8) or 47 x 11 = 517 (P=4) tiles for 256 persistent
    # workgroups -- several tiles per workgroup (next-tile prefetch and commit, the
    # XCD tile permutation); ragged right and bottom edges
    img = oracle.random_image(3000, 700)
    guide = np.ascontiguousarray(img[::-1])
    got = _bilateral_gpu(dev, img, k, guide=guide)
    spans = [(0, 8), (60, 8), (380, 8), (692, 8)]
    want = oracle.bands(lambda r0, n: oracle.joint_bilateral_rows(img, guide, r0, n, k), spans)
    for (r0, n), w_ in zip(spans, want):
        assert np.array_equal(got[r0:r0 + n], w_), (r0, _mismatch(got[r0:r0 + n], w_))


@pytest.mark.parametrize("k", [3, 9, 15, 17, 31])
@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_adaptive(dev, oracle, k, numerics, profile):
    img = oracle.random_image(50, 50)
    h, w, _ = img.shape
    f = vip.CudaAdaptiveBilateralFilter(w, h, k, numerics=numerics)
    d_dst = dev.empty((h, w, 3))
    f.execute(dev.put(img), d_dst)
    got, want = dev.get(d_dst), oracle.adaptive(img, k, profile=profile)
    assert np.array_equal(got, want), _mismatch(got, want)


@pytest.mark.parametrize("k", [5, 15, 17, 19])
def test_adaptive_multi_tile(dev, oracle, k):
    # 3000 x 701: 47 x 11 = 517 tiles of 64 x 64 for 256 persistent workgroups, so
    # every workgroup runs the next-tile prefetch/commit and reuses its LDS sums;
    # ragged edges. k <= 17 takes the separable box-sum path (17: R|B sums unpacked
    # before the horizontal windows), 19 the per-thread square sums
    img = oracle.random_image(3000, 701)
    h, w, _ = img.shape
    f = vip.CudaAdaptiveBilateralFilter(w, h, k)
    d_dst = dev.empty((h, w, 3))
    f.execute(dev.put(img), d_dst)
    got = dev.get(d_dst)
    spans = [(0, 8), (60, 8), (380, 8), (693, 8)]
    want = oracle.bands(lambda r0, n: oracle.adaptive_rows(img, r0, n, k), spans)
    for (r0, n), w_ in zip(spans, want):
        assert np.array_equal(got[r0:r0 + n], w_), (r0, _mismatch(got[r0:r0 + n], w_))


def test_adaptive_natural_image(dev, oracle, lenna):
    h, w, _ = lenna.shape
    f = vip.CudaAdaptiveBilateralFilter(w, h, 15)
    d_dst = dev.empty((h, w, 3))
    f.execute(dev.put(lenna), d_dst)
    got, want = dev.get(d_dst), oracle.adaptive(lenna, 15, threads=16)
    assert np.array_equal(got, want), _mismatch(got, want)


@pytest.mark.parametrize("ch", [1, 3])
@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_gradient(dev, oracle, ch, numerics, profile):
    for src in (oracle.random_u8(2500 * ch).reshape(50, 50, ch), oracle.random_f32(2500 * ch).reshape(50, 50, ch)):
        d_dst = dev.empty((50, 50), np.float32)
        vip.cuda_gradient(dev.put(src), d_dst, 50, 50, ch, numerics=numerics)
        got, want = dev.get(d_dst), oracle.gradient(src, profile)
        assert np.array_equal(got, want), _mismatch(got, want)


@pytest.mark.parametrize("k", [4, 5, 9])
@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_texture_stages_reference_inputs(dev, oracle, k, numerics, profile):
    """test/bilateral_texture_filter.cu:386-461 inputs; blur/rtv bit-exact, guide exact."""
    img = oracle.random_image(50, 50)
    mag = oracle.random_f32(2500).reshape(50, 50)
    t = _TextureImpl(50, 50, k, 1, numerics)
    d_b, d_r = dev.empty((50, 50, 3), np.float32), dev.empty((50, 50), np.float32)
    t.compute_blur_and_rtv(dev.put(img), dev.put(mag), d_b, d_r)
    wb, wr = oracle.blur_rtv(img, mag, k, profile)
    assert np.array_equal(dev.get(d_b), wb)
    assert np.array_equal(dev.get(d_r), wr)
    blurred = oracle.random_f32(7500).reshape(50, 50, 3)
    rtv = oracle.random_f32(2500, 1.0).reshape(50, 50)
    d_g = dev.empty((50, 50, 3))
    t.compute_guide(dev.put(blurred), dev.put(rtv), d_g)
    got, want = dev.get(d_g), oracle.guide(blurred, rtv, k, profile)
    assert np.array_equal(got, want), _mismatch(got, want)


@pytest.mark.parametrize("shape,k,nitr", [((48, 64), 5, 5), ((50, 50), 9, 3), ((121, 203), 5, 3), ((7, 9), 3, 2),
                                           ((40, 70), 4, 2), ((33, 65), 16, 1), ((90, 130), 15, 2)])
@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_texture_end_to_end(dev, oracle, shape, k, nitr, numerics, profile):
    h, w = shape
    img = oracle.random_u8(h * w * 3).reshape(h, w, 3)
    f = vip.CudaBilateralTextureFilter(w, h, k, nitr, numerics=numerics)
    d_dst = dev.empty((h, w, 3))
    f.execute(dev.put(img), d_dst)
    got, want = dev.get(d_dst), oracle.texture(img, k, nitr, profile)
    assert np.array_equal(got, want), _mismatch(got, want)


# FUSED mode (include/vip.h vip_texture_set_mode): guide + JBF of an iteration in one
# launch, the guide kept in LDS; k = 5 only. Ragged shapes cross every tile border case
# (plane positions outside the frame on each side, partial tiles, one-tile frames).
@pytest.mark.parametrize("shape,nitr", [((48, 64), 5), ((50, 50), 3), ((121, 203), 3), ((7, 9), 2), ((1, 1), 1),
                                        ((65, 129), 2), ((200, 300), 2), ((530, 700), 1)])
@pytest.mark.parametrize("numerics,profile", PROFILES)
def test_texture_fused_mode(dev, oracle, shape, nitr, numerics, profile):
    h, w = shape
    img = oracle.random_u8(h * w * 3).reshape(h, w, 3)
    t = _TextureImpl(w, h, 5, nitr, numerics)
    t.set_mode(_TextureImpl.FUSED)
    d_dst = dev.empty((h, w, 3))
    t.execute(dev.put(img), d_dst)
    got, want = dev.get(d_dst), oracle.texture(img, 5, nitr, profile)
    assert np.array_equal(got, want), _mismatch(got, want)
    d = dev.put(img)  # in place
    t.execute(d, d)
    assert np.array_equal(dev.get(d), want)


def test_texture_fused_mode_errors(dev):
    t = _TextureImpl(64, 48, 9, 1)
    with pytest.raises(vip.VipError):  # fused is ksize 5 only
        t.set_mode(_TextureImpl.FUSED)
    with pytest.raises(vip.VipError):
        _TextureImpl(64, 48, 5, 1).set_mode(7)


def test_texture_in_place_and_zero_iterations(dev, oracle):
    img = oracle.random_image(40, 30)
    f = vip.CudaBilateralTextureFilter(40, 30, 5, 1)
    d = dev.put(img)
    f.execute(d, d)  # src == dst is allowed (the reference copied first)
    assert np.array_equal(dev.get(d), oracle.texture(img, 5, 1))
    f0 = vip.CudaBilateralTextureFilter(40, 30, 5, 0)
    d_dst = dev.empty((30, 40, 3))
    f0.execute(dev.put(img), d_dst)
    assert np.array_equal(dev.get(d_dst), img)


def test_lenna_c1_bilateral(dev, oracle, goldens, lenna):
    """BASELINE config C1 (bilateral r=5 on lenna) through the GPU path, both profiles."""
    import hashlib
    for numerics, tag in ((0, "cuda"), (1, "cpp")):
        got = _bilateral_gpu(dev, lenna, 11, numerics=numerics)
        sha = np.frombuffer(hashlib.sha256(got.tobytes()).digest(), np.uint8)
        assert np.array_equal(sha, goldens[f"lenna_bilateral_{tag}_k11_sha256"])


def test_row_band_api_matches_full_frame(dev, oracle):
    """vip_bilateral_run_rows on a band with clamped halo == those rows of the frame."""
    img = oracle.random_image(200, 90)
    full = oracle.bilateral(img, 15)
    impl = _BilateralImpl(200, 90, 15)
    r = 7
    for (b0, b1) in ((0, 30), (30, 61), (61, 90)):
        lo, hi = max(b0 - r, 0), min(b1 + r, 90)
        slab = dev.put(img[lo:hi])
        out = dev.empty((b1 - b0, 200, 3))
        impl.run_rows(slab, out, b1 - b0, b0 - lo, 0, hi - lo)
        assert np.array_equal(dev.get(out), full[b0:b1])
    ada = _AdaptiveImpl(200, 90, 15)
    afull = oracle.adaptive(img, 15)
    slab = dev.put(img[23:77])
    out = dev.empty((40, 200, 3))
    ada.run_rows(slab, out, 40, 7, 0, 54)
    assert np.array_equal(dev.get(out), afull[30:70])


def test_pitched_buffers(dev, oracle):
    """The C ABI takes row pitches; the reference's dense API is pitch = width*3."""
    import ctypes
    img = oracle.random_image(100, 40)
    pitch = 512
    src = np.zeros((40, pitch), np.uint8)
    src[:, :300] = img.reshape(40, 300)
    d_src, d_dst = dev.put(src), dev.empty((40, pitch))
    impl = _BilateralImpl(100, 40, 9)
    vip.lib()  # loaded
    from various_image_processings_amd._lib import call
    call("vip_bilateral_run", impl._h, d_src.data_ptr(), pitch, d_dst.data_ptr(), pitch, None)
    got = dev.get(d_dst)[:, :300].reshape(40, 100, 3)
    assert np.array_equal(got, oracle.bilateral(img, 9))


def test_argument_errors(dev):
    with pytest.raises(vip.VipError) as e:
        vip.CudaBilateralFilter(10, 10, 8)
    assert e.value.code == 10002
    with pytest.raises(vip.VipError):
        vip.CudaBilateralFilter(10, 10, 67)
    f = vip.CudaBilateralFilter(10, 10, 3)
    d = dev.empty((10, 10, 3))
    with pytest.raises(vip.VipError) as e:
        f.bilateral_filter(d, d)
    assert e.value.code == 10003


def test_full_4k_frame_rows_exact(dev, oracle):
    """C2 frame size (3840x2160, r=7): exact on rows spanning both borders and tile seams."""
    img = oracle.random_image(3840, 2160)
    got = _bilateral_gpu(dev, img, 15)
    for r0 in (0, 5, 63, 64, 1000, 2151):
        rows = min(9, 2160 - r0)
        want = oracle.bilateral_rows(img, r0, rows, 15)
        assert np.array_equal(got[r0:r0 + rows], want), (r0, _mismatch(got[r0:r0 + rows], want))


@pytest.mark.parametrize("image", ["random_array_50x50", "lenna"])
def test_profiles_within_reference_tolerance(dev, oracle, lenna, image):
    """GPU output (default CUDA numerics) vs the include/cpp restatement (oracle CPP
    profile) for every filter: within the reference tests' +-1
    (test/bilateral_filter.cu:58-60) for bilateral / joint / adaptive, and <= 1 on
    >= 99.9 % of channels for the iterated texture filter. Prints
    max |delta| and the exact-match percentage (table: DESIGN.md section 2)."""
    img = oracle.random_image(50, 50) if image != "lenna" else lenna
    h, w, _ = img.shape
    guide = np.ascontiguousarray(img[::-1, ::-1])
    d_src, d_dst = dev.put(img), dev.empty(img.shape)
    runs = {
        "bilateral k15": (lambda: vip.CudaBilateralFilter(w, h, 15).bilateral_filter(d_src, d_dst),
                          lambda: oracle.bilateral(img, 15, profile=1, threads=16)),
        "joint k9": (lambda: vip.CudaBilateralFilter(w, h, 9).joint_bilateral_filter(d_src, dev.put(guide), d_dst),
                     lambda: oracle.joint_bilateral(img, guide, 9, profile=1, threads=16)),
        "adaptive k15": (lambda: vip.CudaAdaptiveBilateralFilter(w, h, 15).execute(d_src, d_dst),
                         lambda: oracle.adaptive(img, 15, profile=1, threads=16)),
        "texture k5 nitr5": (lambda: vip.CudaBilateralTextureFilter(w, h, 5, 5).execute(d_src, d_dst),
                             lambda: oracle.texture(img, 5, 5, profile=1)),
    }
    for name, (gpu, cpp) in runs.items():
        gpu()
        diff = np.abs(dev.get(d_dst).astype(int) - cpp().astype(int))
        print(f"{image} {name}: max |delta| {diff.max()}, exact {(diff == 0).mean() * 100:.5f} %, "
              f"<=1 {(diff <= 1).mean() * 100:.5f} %")
        if name.startswith("texture"):
            assert (diff <= 1).mean() >= 0.999, name
        else:
            assert diff.max() <= 1, name


def test_host_frame_async_path(dev, oracle):
    """Pinned host frame -> vip_upload_async -> bilateral on a vip_stream_create stream
    -> vip_download_async: the stream-ordered host path gives the
    same bytes as the oracle."""
    import ctypes
    from various_image_processings_amd._lib import call, lib
    img = oracle.random_image(301, 123)
    n = img.nbytes
    h_in, h_out, stream = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    call("vip_host_alloc", ctypes.byref(h_in), n)
    call("vip_host_alloc", ctypes.byref(h_out), n)
    call("vip_stream_create", ctypes.byref(stream))
    try:
        ctypes.memmove(h_in.value, img.ctypes.data, n)
        ctypes.memset(h_out.value, 0, n)
        d_src, d_dst = dev.empty(img.shape), dev.empty(img.shape)
        f = _BilateralImpl(301, 123, 9)
        call("vip_upload_async", ctypes.c_void_p(d_src.data_ptr()), h_in, n, stream)
        f.bilateral_filter(d_src, d_dst, stream=stream.value)
        call("vip_download_async", h_out, ctypes.c_void_p(d_dst.data_ptr()), n, stream)
        call("vip_stream_synchronize", stream)
        got = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(h_out.value)).reshape(img.shape).copy()
    finally:
        call("vip_stream_destroy", stream)
        call("vip_host_free", h_in)
        call("vip_host_free", h_out)
    want = oracle.bilateral(img, 9)
    assert np.array_equal(got, want), _mismatch(got, want)


def test_split_stream_host_pipeline(dev, oracle):
    """Upload, filter and download on three streams ordered by vip_event_* (the split
    host-frame pipeline of samples/vip_host_pipeline.cpp): same bytes as the oracle."""
    import ctypes
    from various_image_processings_amd._lib import call
    img = oracle.random_image(257, 99)
    n = img.nbytes
    h_in, h_out = ctypes.c_void_p(), ctypes.c_void_p()
    st = [ctypes.c_void_p() for _ in range(3)]
    ev = [ctypes.c_void_p() for _ in range(3)]
    call("vip_host_alloc", ctypes.byref(h_in), n)
    call("vip_host_alloc", ctypes.byref(h_out), n)
    for x in st:
        call("vip_stream_create", ctypes.byref(x))
    for x in ev:
        call("vip_event_create", ctypes.byref(x))
    try:
        ctypes.memmove(h_in.value, img.ctypes.data, n)
        ctypes.memset(h_out.value, 0, n)
        d_src, d_dst = dev.empty(img.shape), dev.empty(img.shape)
        f = _BilateralImpl(257, 99, 15)
        su, sc, sd = st
        call("vip_upload_async", ctypes.c_void_p(d_src.data_ptr()), h_in, n, su)
        call("vip_event_record", ev[0], su)
        call("vip_stream_wait_event", sc, ev[0])
        f.bilateral_filter(d_src, d_dst, stream=sc.value)
        call("vip_event_record", ev[1], sc)
        call("vip_stream_wait_event", sd, ev[1])
        call("vip_download_async", h_out, ctypes.c_void_p(d_dst.data_ptr()), n, sd)
        call("vip_event_record", ev[2], sd)
        call("vip_event_synchronize", ev[2])
        got = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(h_out.value)).reshape(img.shape).copy()
    finally:
        for x in ev:
            call("vip_event_destroy", x)
        for x in st:
            call("vip_stream_destroy", x)
        call("vip_host_free", h_in)
        call("vip_host_free", h_out)
    want = oracle.bilateral(img, 15)
    assert np.array_equal(got, want), _mismatch(got, want)


def _fill_slab(dev, frame, geo):
    """The slab a rank holds after exchange_halo: own rows plus neighbour halo rows."""
    import torch
    b, e = geo.rows
    r = geo.radius
    slab = np.zeros((geo.slab_rows, frame.shape[1], 3), np.uint8)
    slab[r:r + geo.own] = frame[b:e]
    if geo.has_above:
        slab[:r] = frame[b - r:b]
    if geo.has_below:
        slab[r + geo.own:] = frame[e:e + r]
    return dev.put(slab)


@pytest.mark.parametrize("world,shape,k,nitr,numerics", [(3, (100, 70), 5, 3, 0), (2, (64, 130), 3, 5, 1),
                                                         (4, (201, 67), 5, 2, 0), (1, (40, 33), 5, 5, 0)])
def test_sharded_texture_matches_full_frame(dev, oracle, world, shape, k, nitr, numerics):
    """ShardedTexture (one halo exchange of nitr * texture_halo_rows(k) rows, then
    shrinking ghost zones through vip_texture_iterate_rows) on every rank's slab ==
    the full-frame texture filter."""
    from various_image_processings_amd.sharded import ShardedTexture
    h, w = shape
    frame = oracle.random_image(w, h)
    parts = []
    for rank in range(world):
        st = ShardedTexture(w, h, k, nitr, rank, world, numerics=numerics)
        slab = _fill_slab(dev, frame, st.geo)
        out = dev.empty((st.geo.own, w, 3))
        st.filter(slab, out, exchange=False)
        parts.append(dev.get(out))
    got = np.concatenate(parts, axis=0)
    want = oracle.texture(frame, k, nitr, profile=numerics)
    assert np.array_equal(got, want), _mismatch(got, want)


def test_texture_iterate_rows_band(dev, oracle):
    """One vip_texture_iterate_rows call over a middle row band of a whole frame
    (valid rows = the frame) == those rows of a one-iteration texture filter."""
    h, w, k = 90, 77, 5
    frame = oracle.random_image(w, h)
    f = _TextureImpl(w, h, k, 1)
    d_src = dev.put(frame)
    band = dev.empty((31, w, 3))
    f.iterate_rows(d_src, band, 40, 31, 0, h)
    want = oracle.texture(frame, k, 1)
    got = dev.get(band)
    assert np.array_equal(got, want[40:71]), _mismatch(got, want[40:71])


def test_epilogue_division_exact():
    """The bilateral/joint epilogue divides by sumk via one reciprocal (vip_stencil.hpp
    recip_exact/div_by_sumk). microbench/div_check checks RN(1/k) for EVERY float k in
    [1, 2^38) (the epilogue's sums of weights and the texture guide's 1 + exp(x) at every
    ksize) and 2^30 quotients against the IEEE divide on the GPU, the texture
    gradient's sqrt_int_exact against sqrtf for every integer in [0, 2^20), the guide
    blend's pack_u8_clamped against the clamp for every float |v| < 2048, and the rtv
    quotient (rtv_quotient) against the IEEE double divide on 2^30 inputs, half of them at
    float rounding midpoints."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "..", "microbench", "div_check")
    assert os.path.exists(exe), "build first: make -C various_image_processings_amd/csrc"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(" 0 mismatches") == 6, r.stdout


@pytest.mark.parametrize("k,ss,sc", [(31, 1000.0, 1000.0), (5, 0.1, 0.1), (15, 3.0, 1e4), (7, 1e4, 0.5)])
def test_bilateral_extreme_sigmas(dev, oracle, k, ss, sc):
    """sumk at both ends of [1, 961]: flat weights (every tap ~1) and a lone centre tap."""
    img = oracle.random_image(96, 80)
    for guide in (None, np.ascontiguousarray(img[::-1, ::-1])):
        got = _bilateral_gpu(dev, img, k, ss, sc, guide=guide)
        want = oracle.bilateral(img, k, ss, sc) if guide is None else oracle.joint_bilateral(img, guide, k, ss, sc)
        assert np.array_equal(got, want), _mismatch(got, want)


def test_texture_run_timed_matches_execute(dev, oracle):
    """vip_texture_run_timed (the bench's per-stage timing entry point) produces the same
    bytes as vip_texture_run and records 2 * nitr + 1 ordered events."""
    import torch
    img = oracle.random_image(200, 150)
    t = _TextureImpl(200, 150, 5, 3)
    d_src, a, b = dev.put(img), dev.empty(img.shape), dev.empty(img.shape)
    t.execute(d_src, a)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(7)]
    t.execute_timed(d_src, b, ev)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert np.array_equal(dev.get(b), oracle.texture(img, 5, 3))
    assert all(ev[i].elapsed_time(ev[i + 1]) >= 0 for i in range(6))
    with pytest.raises(ValueError):
        t.execute_timed(d_src, b, ev[:6])


def test_device_buffer_validation(dev):
    """filters._ptr rejects wrong dtype, short buffers and host tensors with a Python
    error instead of handing the kernels out-of-bounds pointers."""
    import torch
    f = vip.CudaBilateralFilter(64, 32, 9)
    good = dev.empty((32, 64, 3))
    with pytest.raises(ValueError):
        f.bilateral_filter(dev.empty((31, 64, 3)), good)           # too few rows
    with pytest.raises(ValueError):
        f.bilateral_filter(torch.zeros((32, 64, 3), dtype=torch.float32, device="cuda"), good)  # dtype
    with pytest.raises(ValueError):
        f.bilateral_filter(torch.zeros((32, 64, 3), dtype=torch.uint8), good)  # host tensor
    with pytest.raises(ValueError):
        f.bilateral_filter(dev.empty((32, 128, 3))[:, ::2], good)  # not dense
    impl = _BilateralImpl(64, 32, 9)
    with pytest.raises(vip.VipError):  # C ABI: row range outside the handle's rows
        impl.run_rows(dev.empty((40, 64, 3)), good, 8, 0, 0, 40)
    # DeviceImage carries its dtype: a float32 image is not a u8 frame
    f32img = vip.DeviceImage(64, 32, 3, "float32")
    with pytest.raises(ValueError):
        f.bilateral_filter(f32img, good)


def test_gradient_takes_dtype_from_device_image(dev, oracle):
    """cuda_gradient picks the f32 kernel for a float32 DeviceImage (the reference's
    template argument T), not the u8 one."""
    src = oracle.random_f32(40 * 30 * 3).reshape(30, 40, 3)
    d_src = vip.DeviceImage(40, 30, 3, "float32")
    d_src.upload(src)
    d_dst = vip.DeviceImage(40, 30, 1, "float32")
    vip.cuda_gradient(d_src, d_dst, 40, 30, 3)
    vip.device_synchronize()
    got = np.empty((30, 40), np.float32)
    d_dst.download(got)
    assert np.array_equal(got, oracle.gradient(src))


@pytest.mark.parametrize("kind", ["bilateral", "adaptive", "texture"])
def test_frames_in_flight_on_two_streams(dev, oracle, kind):
    """bench.py's mode: frames i = 0..5 alternate over two HIP streams with no sync
    between them (one handle per stream for the texture filter, which owns scratch
    frames; one shared handle otherwise) -- every output equals the oracle."""
    torch = dev.torch_
    h, w = 360, 640
    imgs = [np.random.default_rng(100 + i).integers(0, 255, (h, w, 3), dtype=np.uint8) for i in range(6)]
    srcs = [dev.put(a) for a in imgs]
    dsts = [dev.empty((h, w, 3)) for _ in imgs]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    if kind == "bilateral":
        f = _BilateralImpl(w, h, 15)
        hs = [lambda s, d, st: f.bilateral_filter(s, d, stream=st)] * 2
        want = [oracle.bilateral(a, 15) for a in imgs]
    elif kind == "adaptive":
        f = _AdaptiveImpl(w, h, 15)
        hs = [lambda s, d, st: f.execute(s, d, stream=st)] * 2
        want = [oracle.adaptive(a, 15) for a in imgs]
    else:
        ts = [_TextureImpl(w, h, 5, 3) for _ in range(2)]
        hs = [lambda s, d, st, t=t: t.execute(s, d, stream=st) for t in ts]
        want = [oracle.texture(a, 5, 3) for a in imgs]
    for i in range(6):
        hs[i % 2](srcs[i], dsts[i], streams[i % 2])
    for i in range(6):
        got = dev.get(dsts[i])
        assert np.array_equal(got, want[i]), f"frame {i}: " + _mismatch(got, want[i])


def test_launched_kernels_names_the_instantiation(dev, oracle):
    """vip_launched_kernels: the exact template instantiation of each launch, as rocprofv3
    names it (profiles/r03_c2_busy.json holds the C2 one), each once, cleared per call."""
    vip.launched_kernels()
    img = oracle.random_image(3840, 2160)
    d = dev.empty((2160, 3840, 3))
    f = vip.CudaBilateralFilter(3840, 2160, 15)
    f.bilateral_filter(dev.put(img), d)
    f.bilateral_filter(dev.put(img), d)
    assert vip.launched_kernels() == ["void vip::bilateral_kernel<7, 16, false, true, 32, 8, 768, false, 16, false>"]
    assert vip.launched_kernels() == []
    vip.CudaBilateralTextureFilter(300, 200, 5, 2).execute(dev.put(img[:200, :300].copy()), dev.empty((200, 300, 3)))
    names = vip.launched_kernels()
    assert len(names) == 2 and any(n.startswith("void vip::texture_guide_fused_kernel<2, false>") for n in names)
    assert all("(" not in n for n in names)


def test_kernel_timing_stamps_each_launch(dev, oracle):
    """vip_kernel_timing: each launch inside the window carries kernel-stamped events (its
    own begin and end, hipExtLaunchKernel); launches beyond the capacity run plainly; the
    outputs are the same as without the recorder."""
    img = oracle.random_image(640, 360)
    d = dev.empty((360, 640, 3))
    f = vip.CudaBilateralFilter(640, 360, 15)
    with vip.kernel_timing(3) as kt:
        for _ in range(5):
            f.bilateral_filter(dev.put(img), d)
    assert kt.count == 3
    rec = kt.records()
    assert all(n.startswith("void vip::bilateral_kernel<7,") for n, _ in rec)
    assert all(0.0 < ms < 100.0 for _, ms in rec)
    assert np.array_equal(dev.get(d), oracle.bilateral(img, 15, threads=16))
    t = _TextureImpl(300, 200, 5, 2)
    with vip.kernel_timing(16) as kt:
        t.execute(dev.put(img[:200, :300].copy()), dev.empty((200, 300, 3)))
    dur = kt.durations()
    assert kt.count == 4 and sum(len(v) for v in dur.values()) == 4
    assert any(n.startswith("void vip::texture_guide_fused_kernel<2, false>") for n in dur)
    with pytest.raises(vip.VipError):
        vip.kernel_timing(0).__enter__()


def test_kernel_timing_leaves_captured_launches_plain(dev, oracle):
    """A launch captured into a graph while the recorder is on takes no events (they would
    never be stamped): the recorder counts nothing and the replayed graph filters exactly."""
    from various_image_processings_amd.filters import _BilateralImpl
    torch = dev.torch_
    img = oracle.random_image(256, 128)
    src, dst = dev.put(img), dev.empty((128, 256, 3))
    b = _BilateralImpl(256, 128, 9)
    s = torch.cuda.Stream()
    b.bilateral_filter(src, dst, stream=s)  # first launch (LDS attribute) outside the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with vip.kernel_timing(4) as kt:
        with torch.cuda.graph(g, stream=s):
            b.bilateral_filter(src, dst, stream=s)
    assert kt.count == 0
    dst.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(dev.get(dst), oracle.bilateral(img, 9))


def test_small_frame_tiling_follows_frames_in_flight(dev, oracle):
    """The plain kernel's small-frame tiling counts the frames in flight (distinct streams
    among the device's last 8 launches): lenna-sized 512^2 frames on 4 streams take the
    throughput tiling (16-wave 256-pixel tiles, 64 per frame: four frames side by side), one
    stream the latency tiling (4-wave 256-pixel tiles). Same bytes either way."""
    from various_image_processings_amd.filters import _BilateralImpl
    torch = dev.torch_
    img = oracle.random_image(512, 512)
    src = dev.put(img)
    want = oracle.bilateral(img, 11, threads=16)
    impl = _BilateralImpl(512, 512, 11)
    streams = [torch.cuda.Stream() for _ in range(4)]
    outs = [dev.empty((512, 512, 3)) for _ in streams]
    for _ in range(3):  # fill the ring with the 4 streams
        for s, o in zip(streams, outs):
            impl.bilateral_filter(src, o, stream=s)
    torch.cuda.synchronize()
    vip.launched_kernels()
    for _ in range(2):
        for s, o in zip(streams, outs):
            impl.bilateral_filter(src, o, stream=s)
    torch.cuda.synchronize()
    assert vip.launched_kernels() == ["void vip::bilateral_kernel<5, 16, false, true, 32, 4, 768, false, 64, false>"]
    for o in outs:
        assert np.array_equal(dev.get(o), want)
    for _ in range(8):  # one stream only: the ring forgets the others
        impl.bilateral_filter(src, outs[0], stream=streams[0])
    torch.cuda.synchronize()
    vip.launched_kernels()
    impl.bilateral_filter(src, outs[1], stream=streams[0])
    torch.cuda.synchronize()
    assert vip.launched_kernels() == ["void vip::bilateral_kernel<5, 4, false, true, 32, 4, 768, false, 64, false>"]
    assert np.array_equal(dev.get(outs[0]), want) and np.array_equal(dev.get(outs[1]), want)
    vip.set_bilateral_frames_in_flight(4)  # the measurement override: one stream, the in-flight tiling
    try:
        impl.bilateral_filter(src, outs[2], stream=streams[0])
        torch.cuda.synchronize()
    finally:
        vip.set_bilateral_frames_in_flight(0)
    assert vip.launched_kernels() == ["void vip::bilateral_kernel<5, 16, false, true, 32, 4, 768, false, 64, false>"]
    assert np.array_equal(dev.get(outs[2]), want)
    with pytest.raises(vip.VipError):
        vip.set_bilateral_frames_in_flight(5)
