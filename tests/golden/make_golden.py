"""Regenerate tests/golden/ (run in the dev container, where /root/reference exists).

1. random_array_*.bin — outputs of the reference's OWN input generator
   (test/random_array.hpp, compiled in place by oracle/Makefile into
   oracle/_ref/random_array_dump). These pin the oracle's mt19937 restatement.
2. lenna_bgr.npz — sample_image/lenna.png decoded as cv::imread(IMREAD_COLOR)
   would (RGBA -> BGR, alpha dropped); the C1 plumbing input.
3. oracle_*.npz — oracle outputs on the reference tests' inputs (regression
   anchors for the CPU oracle; the GPU tests recompute the oracle live as well).
"""
import hashlib
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle as o  # noqa: E402

REF_DUMP = os.path.join(ROOT, "oracle", "_ref", "random_array_dump")


def ref_random(kind, n, mx):
    return subprocess.run([REF_DUMP, kind, str(n), str(mx)], check=True, capture_output=True).stdout


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    # (1) reference generator outputs, the exact calls of the reference tests
    fixtures = {
        "random_array_u8_7500_255.bin": ("u8", 7500, 255),     # 50x50x3 images (every filter test)
        "random_array_u8_2500_255.bin": ("u8", 2500, 255),     # gradient 1ch
        "random_array_f32_2500_255.bin": ("f32", 2500, 255),   # magnitude / gradient f32
        "random_array_f32_7500_255.bin": ("f32", 7500, 255),   # blurred (guide test), gradient f32 3ch
        "random_array_f32_2500_1.bin": ("f32", 2500, 1),       # rtv (guide test)
    }
    for name, (kind, n, mx) in fixtures.items():
        with open(os.path.join(HERE, name), "wb") as f:
            f.write(ref_random(kind, n, mx))

    # (2) lenna as BGR
    from PIL import Image
    rgba = np.asarray(Image.open("/root/reference/sample_image/lenna.png").convert("RGBA"))
    bgr = np.ascontiguousarray(rgba[..., [2, 1, 0]])
    np.savez_compressed(os.path.join(HERE, "lenna_bgr.npz"), bgr=bgr)

    # (3) oracle outputs on the reference tests' inputs
    img = o.random_image(50, 50)
    out = {}
    for prof, tag in ((o.CUDA, "cuda"), (o.CPP, "cpp")):
        for k in (3, 9, 11, 15, 31):
            out[f"bilateral_{tag}_k{k}"] = o.bilateral(img, k, 10.0, 30.0, prof)
            out[f"adaptive_{tag}_k{k}"] = o.adaptive(img, k, 10.0, 30.0, prof)
        guide_img = o.random_u8(7500)[::-1].copy().reshape(50, 50, 3)
        out[f"joint_{tag}_k9"] = o.joint_bilateral(img, guide_img, 9, 10.0, 30.0, prof)
        mag = o.random_f32(2500).reshape(50, 50)
        for k in (5, 9):
            b, r = o.blur_rtv(img, mag, k, prof)
            out[f"blurred_{tag}_k{k}"] = b
            out[f"rtv_{tag}_k{k}"] = r
            out[f"guide_{tag}_k{k}"] = o.guide(o.random_f32(7500).reshape(50, 50, 3),
                                               o.random_f32(2500, 1.0).reshape(50, 50), k, prof)
        for ch in (1, 3):
            out[f"gradient_u8_{tag}_c{ch}"] = o.gradient(o.random_u8(2500 * ch).reshape(50, 50, ch), prof)
            out[f"gradient_f32_{tag}_c{ch}"] = o.gradient(o.random_f32(2500 * ch).reshape(50, 50, ch), prof)
        out[f"texture_{tag}_k5_n5"] = o.texture(o.random_image(64, 48), 5, 5, prof)
        lenna_k11 = o.bilateral(bgr, 11, 10.0, 30.0, prof)
        out[f"lenna_bilateral_{tag}_k11_sha256"] = np.frombuffer(
            hashlib.sha256(lenna_k11.tobytes()).digest(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "oracle_small.npz"), **out)
    print("wrote", len(fixtures), "reference fixtures and", len(out), "oracle goldens")


if __name__ == "__main__":
    main()
