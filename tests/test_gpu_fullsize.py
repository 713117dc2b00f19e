"""Every BASELINE.json GPU config at its own frame size, bit-exact against the oracle.

The HIP path filters the whole frame in one call (the persistent kernels then run
several tiles per workgroup: 1,020 bilateral tiles on 256 CUs at 4K, 16,512 at
16384^2); the oracle recomputes row bands that cross the top and bottom frame
borders, tile seams (64-row tiles) and, with full-width rows, every column seam and
both side borders. Bands are independent, so they run in parallel threads.

  C2 bilateral r=7 3840x2160           (also tests/test_gpu_parity.py::test_full_4k_frame_rows_exact)
  C3 adaptive r=7 3840x2160            test_c3_adaptive_4k
  C4 texture k=5 nitr=5 3840x2160      test_c4_texture_4k (bands on crops with a 45-row ghost margin)
  C5 bilateral r=15 16384x16384        test_c5_bilateral_16k_single_launch_and_8_way_split
  C3 / C4 frames split 8 ways          test_4k_8_way_split_equals_single_launch
References: src/adaptive_bilateral_filter_impl.cu:7-115,
src/bilateral_texture_filter_impl.cu:199-214, src/bilateral_filter_impl.cu:7-96.
"""
import numpy as np
import pytest

import various_image_processings_amd as vip

pytestmark = pytest.mark.gpu

BANDS_4K = [(0, 10), (60, 8), (1020, 9), (2150, 10)]


def _mismatch(a, b):
    d = np.argwhere(a != b)
    return f"{len(d)} mismatches, first {d[:5].tolist()}"


def _check_bands(got_rows, want_rows, spans):
    for (r0, n), g, w in zip(spans, got_rows, want_rows):
        assert np.array_equal(g, w), (r0, n, _mismatch(g, w))


@pytest.mark.parametrize("numerics", [0, 1])
def test_c3_adaptive_4k(dev, oracle, numerics):
    img = oracle.random_image(3840, 2160)
    f = vip.CudaAdaptiveBilateralFilter(3840, 2160, 15, numerics=numerics)
    d_dst = dev.empty(img.shape)
    f.execute(dev.put(img), d_dst)
    got = dev.get(d_dst)
    want = oracle.bands(lambda r0, n: oracle.adaptive_rows(img, r0, n, 15, profile=numerics), BANDS_4K)
    _check_bands([got[r0:r0 + n] for r0, n in BANDS_4K], want, BANDS_4K)


@pytest.mark.parametrize("kind", ["bilateral", "adaptive", "texture"])
def test_reference_defaults_4k_natural_image(dev, oracle, lenna, kind):
    """The reference samples' default parameters (ksize 9, sigma 10 / 30; texture ksize 9,
    nitr 3: sample/*/main.cpp) on a 4K frame of natural-image statistics (lenna tiled,
    SURVEY 8(d) input iii): small colour distances dominate, unlike uniform noise."""
    img = np.ascontiguousarray(np.tile(lenna, (5, 8, 1))[:2160, :3840])
    d_dst = dev.empty(img.shape)
    if kind == "bilateral":
        vip.CudaBilateralFilter(3840, 2160).bilateral_filter(dev.put(img), d_dst)
        fn = lambda r0, n: oracle.bilateral_rows(img, r0, n, 9)  # noqa: E731
    elif kind == "adaptive":
        vip.CudaAdaptiveBilateralFilter(3840, 2160).execute(dev.put(img), d_dst)
        fn = lambda r0, n: oracle.adaptive_rows(img, r0, n, 9)  # noqa: E731
    else:
        vip.CudaBilateralTextureFilter(3840, 2160).execute(dev.put(img), d_dst)
        fn = lambda r0, n: oracle.texture_rows(img, r0, n, 9, 3)  # noqa: E731
    got = dev.get(d_dst)
    spans = [(0, 12), (508, 8), (2148, 12)]
    _check_bands([got[r0:r0 + n] for r0, n in spans], oracle.bands(fn, spans), spans)


@pytest.mark.parametrize("numerics", [0, 1])
def test_c2_bilateral_4k_profiles(dev, oracle, numerics):
    img = oracle.random_image(3840, 2160)
    f = vip.CudaBilateralFilter(3840, 2160, 15, numerics=numerics)
    d_dst = dev.empty(img.shape)
    f.bilateral_filter(dev.put(img), d_dst)
    got = dev.get(d_dst)
    want = oracle.bands(lambda r0, n: oracle.bilateral_rows(img, r0, n, 15, profile=numerics), BANDS_4K)
    _check_bands([got[r0:r0 + n] for r0, n in BANDS_4K], want, BANDS_4K)


@pytest.mark.parametrize("k,ss,sc", [(9, 4.0, 1.73205080757), (25, 10.0, 30.0)])
def test_joint_bilateral_4k(dev, oracle, k, ss, sc):
    """k=9, sigma 4 / sqrt(3) is the texture filter's JBF at k=5 (C4); k=25 takes the
    4-outputs-per-thread joint kernel. Many persistent tiles per workgroup."""
    img = oracle.random_image(3840, 2160)
    guide = np.ascontiguousarray(img[::-1, ::-1])
    f = vip.CudaBilateralFilter(3840, 2160, k, ss, sc)
    d_dst = dev.empty(img.shape)
    f.joint_bilateral_filter(dev.put(img), dev.put(guide), d_dst)
    got = dev.get(d_dst)
    want = oracle.bands(lambda r0, n: oracle.joint_bilateral_rows(img, guide, r0, n, k, ss, sc), BANDS_4K)
    _check_bands([got[r0:r0 + n] for r0, n in BANDS_4K], want, BANDS_4K)


@pytest.mark.parametrize("numerics", [0, 1])
def test_c4_texture_4k(dev, oracle, numerics):
    img = oracle.random_image(3840, 2160)
    f = vip.CudaBilateralTextureFilter(3840, 2160, 5, 5, numerics=numerics)
    d_dst = dev.empty(img.shape)
    f.execute(dev.put(img), d_dst)
    got = dev.get(d_dst)
    spans = [(0, 16), (1016, 24), (2144, 16)]
    want = oracle.bands(lambda r0, n: oracle.texture_rows(img, r0, n, 5, 5, profile=numerics), spans)
    _check_bands([got[r0:r0 + n] for r0, n in spans], want, spans)


@pytest.mark.parametrize("numerics", [0, 1])
def test_c4_texture_4k_fused_equals_two_launch(dev, oracle, numerics):
    """C4 in FUSED mode (guide + JBF per iteration in one launch) equals the two-launch
    pipeline on every pixel of the 4K frame (which test_c4_texture_4k pins to the
    oracle), plus oracle bands of its own."""
    from various_image_processings_amd.filters import _TextureImpl
    img = oracle.random_image(3840, 2160)
    d_src = dev.put(img)
    outs = []
    for mode in (_TextureImpl.TWO_LAUNCH, _TextureImpl.FUSED):
        t = _TextureImpl(3840, 2160, 5, 5, numerics)
        t.set_mode(mode)
        d_dst = dev.empty(img.shape)
        t.execute(d_src, d_dst)
        outs.append(dev.get(d_dst))
    assert np.array_equal(outs[0], outs[1]), "fused != two-launch"
    spans = [(0, 8), (2152, 8)]
    want = oracle.bands(lambda r0, n: oracle.texture_rows(img, r0, n, 5, 5, profile=numerics), spans)
    _check_bands([outs[1][r0:r0 + n] for r0, n in spans], want, spans)


def test_c5_bilateral_16k_single_launch_and_8_way_split(dev, oracle):
    """C5 (r=15, 16384^2): one launch on one GPU, bands against the oracle; then the
    frame split 8 ways through ShardedBilateral (each rank's slab = its 2048 rows
    plus the 15-row halos a real exchange would deliver, clamp range per position)
    must equal the single launch on all 268M pixels."""
    import torch
    from various_image_processings_amd.sharded import ShardedBilateral
    n = 16384
    img = np.random.default_rng(42).integers(0, 255, (n, n, 3), dtype=np.uint8)
    d_src = dev.put(img)
    d_full = dev.empty(img.shape)
    vip.CudaBilateralFilter(n, n, 31).bilateral_filter(d_src, d_full)
    spans = [(0, 9), (2040, 16), (8190, 4), (16375, 9)]
    got = [d_full[r0:r0 + k].cpu().numpy() for r0, k in spans]
    want = oracle.bands(lambda r0, k: oracle.bilateral_rows(img, r0, k, 31), spans)
    _check_bands(got, want, spans)
    del img
    for rank in range(8):
        sb = ShardedBilateral(n, n, 31, rank, 8)
        g = sb.geo
        b, e = g.rows
        r = g.radius
        slab = torch.zeros((g.slab_rows, n, 3), dtype=torch.uint8, device="cuda")
        lo, hi = max(b - r, 0), min(e + r, n)
        slab[r - (b - lo):r + g.own + (hi - e)] = d_src[lo:hi]  # own rows + the neighbours' halo rows
        out = torch.empty((g.own, n, 3), dtype=torch.uint8, device="cuda")
        sb.filter(slab, out, exchange=False)
        torch.cuda.synchronize()
        assert torch.equal(out, d_full[b:e]), f"rank {rank}: {int((out != d_full[b:e]).sum())} bytes differ"


@pytest.mark.parametrize("kind", ["adaptive", "texture"])
def test_4k_8_way_split_equals_single_launch(dev, oracle, kind):
    """SURVEY 8(f)3 at BASELINE size: the C3 / C4 frame split 8 ways (ShardedBilateral
    adaptive with a 7-row halo; ShardedTexture with one 45-row halo per frame and
    shrinking ghost zones) equals the single-GPU launch on every pixel. Each rank's slab
    holds its rows plus the neighbours' halo rows a real exchange would deliver."""
    import torch
    from various_image_processings_amd.sharded import ShardedBilateral, ShardedTexture
    w, h = 3840, 2160
    img = oracle.random_image(w, h)
    d_src = dev.put(img)
    d_full = dev.empty(img.shape)
    if kind == "texture":
        vip.CudaBilateralTextureFilter(w, h, 5, 5).execute(d_src, d_full)
    else:
        vip.CudaAdaptiveBilateralFilter(w, h, 15).execute(d_src, d_full)
    for rank in range(8):
        sh = ShardedTexture(w, h, 5, 5, rank, 8) if kind == "texture" else \
            ShardedBilateral(w, h, 15, rank, 8, adaptive=True)
        g = sh.geo
        b, e = g.rows
        r = g.radius
        slab = torch.zeros((g.slab_rows, w, 3), dtype=torch.uint8, device="cuda")
        lo, hi = max(b - r, 0), min(e + r, h)
        slab[r - (b - lo):r + g.own + (hi - e)] = d_src[lo:hi]
        out = torch.empty((g.own, w, 3), dtype=torch.uint8, device="cuda")
        sh.filter(slab, out, exchange=False)
        torch.cuda.synchronize()
        assert torch.equal(out, d_full[b:e]), f"{kind} rank {rank}: {int((out != d_full[b:e]).sum())} bytes differ"
