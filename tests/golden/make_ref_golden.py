"""Regenerate tests/golden/ref_oracles.npz (run in the dev container, where /root/reference
exists): outputs of the reference tests' OWN CPU oracles, compiled where they lie
(oracle/ref_test_oracles.cpp + oracle/Makefile -> oracle/_ref/libref_test_oracles.so):

  RefAdaptiveBilateralFilterImpl   test/adaptive_bilateral_filter.cu:7-119
  RefBilateralTextureFilterImpl    test/bilateral_texture_filter.cu:8-113 (blur/rtv, guide)
  ref_gradient<T>                  test/gradient.cu:9-34
  internal::pre_compute_kernels    include/cpp/bilateral_filter.hpp:10-39 (the include/cpp LUTs)

on the reference tests' own inputs (test/random_array.hpp, seed 42, 50x50: the inputs every
gtest case of those files builds) at ksize 9 (their default) and 15, plus one 640x360 frame
through the whole texture-stage chain (gradient -> blur/rtv -> guide) and the adaptive filter,
and the adaptive filter on lenna. Small outputs are stored whole; the 640x360 and lenna ones
as sha256 digests (the oracle's REF profile regenerates them bit for bit, which is what the
CPU tests check, and the GPU tests then compare the HIP outputs with those at the
reference's own tolerances). The fixture holds data only, no reference source text.
"""
import hashlib
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

SMALL_K = (9, 15)
# include/cpp LUT sets (ksize, sigma_space, sigma_color, colour LUT length): the bilateral
# defaults, BASELINE C2/C5, the largest ksize, a narrow sigma, and the adaptive filter's 1536
LUT_CASES = ((9, 10.0, 30.0, 768), (15, 10.0, 30.0, 768), (31, 20.0, 60.0, 768), (65, 10.0, 30.0, 768),
             (9, 4.0, 1.73205080757, 768), (15, 10.0, 30.0, 1536), (63, 10.0, 30.0, 1536))
CHAIN_K = (5, 9)
OUT = os.path.join(HERE, "ref_oracles.npz")


def inputs(o):
    """The reference tests' inputs, from the oracle's generator (pinned to
    test/random_array.hpp by tests/golden/random_array_*.bin)."""
    return dict(
        img50=o.random_image(50, 50),                        # every filter test's image
        mag50=o.random_f32(2500).reshape(50, 50),            # CudaComputeBlurAndRTV magnitude
        blur50=o.random_f32(7500).reshape(50, 50, 3),        # CudaComputeGuide blurred
        rtv50=o.random_f32(2500, 1.0).reshape(50, 50),       # CudaComputeGuide rtv (max 1)
        u8c1=o.random_u8(2500).reshape(50, 50, 1), u8c3=o.random_u8(7500).reshape(50, 50, 3),
        f32c1=o.random_f32(2500).reshape(50, 50, 1), f32c3=o.random_f32(7500).reshape(50, 50, 3),
        img640=o.random_image(640, 360),
    )


def sha(a: np.ndarray) -> np.ndarray:
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), np.uint8)


def compute(ref, x, lenna):
    """Every fixture entry from `ref` (the compiled reference oracles, or the oracle's REF
    profile behind the same five functions)."""
    out = {}
    for k in SMALL_K:
        out[f"adaptive_k{k}"] = ref.adaptive(x["img50"], k)
        out[f"blurred_k{k}"], out[f"rtv_k{k}"] = ref.blur_rtv(x["img50"], x["mag50"], k)
        out[f"guide_k{k}"] = ref.guide(x["blur50"], x["rtv50"], k)
    for name in ("u8c1", "u8c3", "f32c1", "f32c3"):
        out[f"gradient_{name}"] = ref.gradient(x[name])
    out["adaptive640_k9_sha256"] = sha(ref.adaptive(x["img640"], 9))
    out["adaptive_lenna_k15_sha256"] = sha(ref.adaptive(lenna, 15))
    mag = ref.gradient(x["img640"])
    out["chain640_magnitude_sha256"] = sha(mag)
    for k in CHAIN_K:
        b, r = ref.blur_rtv(x["img640"], mag, k)
        out[f"chain640_k{k}_blurred_sha256"] = sha(b)
        out[f"chain640_k{k}_rtv_sha256"] = sha(r)
        out[f"chain640_k{k}_guide_sha256"] = sha(ref.guide(b, r, k))
    return out


def compute_luts(luts):
    """luts(ksize, sigma_space, sigma_color, color_len) -> (space, colour), per LUT_CASES."""
    out = {}
    for k, ss, sc, n in LUT_CASES:
        sp, co = luts(k, ss, sc, n)
        out[f"cpp_lut_space_k{k}_s{ss:g}_c{sc:g}_n{n}"] = np.asarray(sp, np.float32).reshape(k, k)
        out[f"cpp_lut_color_k{k}_s{ss:g}_c{sc:g}_n{n}"] = np.asarray(co, np.float32)
    return out


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    from oracle import oracle as o
    from oracle import ref_test_oracles as ref
    if not ref.available():
        raise SystemExit("oracle/_ref/libref_test_oracles.so missing: /root/reference not mounted?")
    lenna = np.load(os.path.join(HERE, "lenna_bgr.npz"))["bgr"]
    out = compute(ref, inputs(o), lenna)
    out.update(compute_luts(ref.cpp_luts))
    np.savez_compressed(OUT, **out)
    print("wrote", len(out), "entries to", os.path.relpath(OUT, ROOT))


if __name__ == "__main__":
    main()
