"""The HIP path against the reference tests' OWN oracles (tests/golden/ref_oracles.npz: the
Ref* classes of test/adaptive_bilateral_filter.cu, test/bilateral_texture_filter.cu and
test/gradient.cu, compiled in place; tests/golden/make_ref_golden.py), at the tolerances the
reference's own CUDA tests apply to its kernels:

  adaptive      +-1 per channel   test/adaptive_bilateral_filter.cu:185-193 (exact share printed)
  blur / rtv    FLOAT_EQ (4 ulp)  test/bilateral_texture_filter.cu:253-262
  guide         EQ                test/bilateral_texture_filter.cu:279-283
  gradient      FLOAT_EQ          test/gradient.cu (CudaRandom* cases)

Frames beyond the fixture's 50x50 arrays (640x360, lenna) compare with the oracle's REF
profile, which tests/test_ref_pinned.py pins to those Ref oracles by sha256.
"""
import os
import sys

import numpy as np
import pytest

import various_image_processings_amd as vip
from conftest import GOLDEN
from various_image_processings_amd.filters import _TextureImpl

sys.path.insert(0, GOLDEN)
import make_ref_golden as mrg  # noqa: E402

pytestmark = pytest.mark.gpu
NUMERICS = [vip.VIP_NUMERICS_CUDA, vip.VIP_NUMERICS_CPP]


@pytest.fixture(scope="module")
def fixture():
    return dict(np.load(os.path.join(GOLDEN, "ref_oracles.npz")))


@pytest.fixture(scope="module")
def inputs(oracle):
    return mrg.inputs(oracle)


def ulps(a, b):
    def key(x):
        i = np.ascontiguousarray(x, np.float32).view(np.int32).astype(np.int64)
        return np.where(i < 0, -(i & 0x7FFFFFFF), i)
    return np.abs(key(a) - key(b))


def _adaptive(dev, img, k, numerics):
    h, w, _ = img.shape
    d_dst = dev.empty((h, w, 3))
    vip.CudaAdaptiveBilateralFilter(w, h, k, numerics=numerics).execute(dev.put(img), d_dst)
    return dev.get(d_dst)


def _near1(got, want, what):
    d = np.abs(got.astype(int) - want.astype(int))
    print(f"{what}: max |d| {d.max()}, exact {100 * (d == 0).mean():.4f} %")
    assert d.max() <= 1, what
    return (d == 0).mean()


@pytest.mark.parametrize("numerics", NUMERICS)
@pytest.mark.parametrize("k", mrg.SMALL_K)
def test_adaptive_vs_reference_oracle(dev, fixture, inputs, k, numerics):
    _near1(_adaptive(dev, inputs["img50"], k, numerics), fixture[f"adaptive_k{k}"], f"adaptive k{k} numerics {numerics}")


@pytest.mark.parametrize("numerics", NUMERICS)
def test_adaptive_vs_reference_oracle_large(dev, oracle, inputs, lenna, numerics):
    for img, k in ((inputs["img640"], 9), (lenna, 15)):
        want = oracle.adaptive(img, k, profile=oracle.REF, threads=16)
        assert _near1(_adaptive(dev, img, k, numerics), want, f"adaptive {img.shape} k{k}") > 0.9999


@pytest.mark.parametrize("numerics", NUMERICS)
@pytest.mark.parametrize("k", mrg.SMALL_K)
def test_texture_stages_vs_reference_oracle(dev, fixture, inputs, k, numerics):
    t = _TextureImpl(50, 50, k, 1, numerics)
    d_b, d_r = dev.empty((50, 50, 3), np.float32), dev.empty((50, 50), np.float32)
    t.compute_blur_and_rtv(dev.put(inputs["img50"]), dev.put(inputs["mag50"]), d_b, d_r)
    assert ulps(dev.get(d_b), fixture[f"blurred_k{k}"]).max() <= 4
    assert ulps(dev.get(d_r), fixture[f"rtv_k{k}"]).max() <= 4
    d_g = dev.empty((50, 50, 3))
    t.compute_guide(dev.put(inputs["blur50"]), dev.put(inputs["rtv50"]), d_g)
    assert np.array_equal(dev.get(d_g), fixture[f"guide_k{k}"])


@pytest.mark.parametrize("numerics", NUMERICS)
@pytest.mark.parametrize("k", mrg.CHAIN_K)
def test_texture_stage_chain_640_vs_reference_oracle(dev, oracle, inputs, k, numerics):
    """Each HIP stage on the Ref chain's own inputs (a 640x360 frame, its Ref gradient, the Ref
    blur/rtv of it): magnitude and blur/rtv FLOAT_EQ, guide EQ."""
    img = inputs["img640"]
    mag = oracle.gradient(img, oracle.REF)
    d_m = dev.empty((360, 640), np.float32)
    vip.cuda_gradient(dev.put(img), d_m, 640, 360, 3, numerics=numerics)
    assert ulps(dev.get(d_m), mag).max() <= 4
    b, r = oracle.blur_rtv(img, mag, k, oracle.REF)
    t = _TextureImpl(640, 360, k, 1, numerics)
    d_b, d_r = dev.empty((360, 640, 3), np.float32), dev.empty((360, 640), np.float32)
    t.compute_blur_and_rtv(dev.put(img), dev.put(mag), d_b, d_r)
    assert ulps(dev.get(d_b), b).max() <= 4
    assert ulps(dev.get(d_r), r).max() <= 4
    d_g = dev.empty((360, 640, 3))
    t.compute_guide(dev.put(b), dev.put(r), d_g)
    assert np.array_equal(dev.get(d_g), oracle.guide(b, r, k, oracle.REF))


@pytest.mark.parametrize("numerics", NUMERICS)
@pytest.mark.parametrize("name", ["u8c1", "u8c3", "f32c1", "f32c3"])
def test_gradient_vs_reference_oracle(dev, fixture, inputs, name, numerics):
    src = inputs[name]
    d_dst = dev.empty((50, 50), np.float32)
    vip.cuda_gradient(dev.put(src), d_dst, 50, 50, src.shape[2], numerics=numerics)
    assert ulps(dev.get(d_dst), fixture[f"gradient_{name}"]).max() <= 4
