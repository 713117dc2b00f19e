"""The reference API's default parameters on a 4K frame (include/cuda/*.hpp defaults: ksize 9,
sigma_space 10, sigma_color 30; texture ksize 9, nitr 3): kernel-stamped duration of each
launch (vip_kernel_timing), mean over 20 calls after a 1 s clock settle, and the in-disc tap
rate where the kernel is a stencil.
usage: python scripts/experiments/defaults_bench.py"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import various_image_processings_amd as vip  # noqa: E402
from various_image_processings_amd.filters import _AdaptiveImpl, _BilateralImpl, _TextureImpl  # noqa: E402

W, H = 3840, 2160
src = [torch.randint(0, 255, (H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(2)]
gd = torch.randint(0, 255, (H, W, 3), dtype=torch.uint8, device="cuda")
dst = torch.empty_like(src[0])


def taps(r):
    return sum(1 for y in range(-r, r + 1) for x in range(-r, r + 1) if x * x + y * y <= r * r)


cases = {
    "bilateral_k9": (lambda i, b=_BilateralImpl(W, H, 9): b.bilateral_filter(src[i % 2], dst), taps(4)),
    "joint_k9": (lambda i, b=_BilateralImpl(W, H, 9): b.joint_bilateral_filter(src[i % 2], gd, dst), taps(4)),
    "adaptive_k9": (lambda i, a=_AdaptiveImpl(W, H, 9): a.execute(src[i % 2], dst), taps(4)),
    "texture_k9_nitr3": (lambda i, t=_TextureImpl(W, H, 9, 3): t.execute(src[i % 2], dst), None),
}
for name, (fn, nt) in cases.items():
    t0, i = time.perf_counter(), 0
    while time.perf_counter() - t0 < 1.0:
        fn(i)
        i += 1
        if i % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    with vip.kernel_timing(256) as kt:
        for j in range(20):
            fn(j)
    d = {n: round(1e3 * sum(v) / len(v), 2) for n, v in kt.durations().items()}
    out = {"case": name, "us_per_launch": d}
    if nt:
        us = sum(d.values())
        out["gtaps_per_s"] = round(nt * W * H / (us * 1e-6) / 1e9, 1)
    print(json.dumps(out), flush=True)
