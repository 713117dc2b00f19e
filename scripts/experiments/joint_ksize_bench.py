"""Joint bilateral filter on a 4K frame at the reference API's default sigmas (space 10,
colour 30: the unfolded colour LUT) for each ksize: kernel-stamped duration per launch,
mean over 20 launches after a 1 s clock settle, the in-disc tap rate, and parity of the
same build against the oracle on a ragged frame.
usage: python scripts/experiments/joint_ksize_bench.py [--lib variants/x.so] [k ...]"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
args = sys.argv[1:]
if args[:1] == ["--lib"]:  # an alternative library build (scripts/build_*variant.sh)
    import various_image_processings_amd._lib as L
    L.LIB_PATH, args = args[1], args[2:]
import various_image_processings_amd as vip  # noqa: E402
from various_image_processings_amd.filters import _BilateralImpl  # noqa: E402

W, H = 3840, 2160
ks = [int(a) for a in args] or [3, 5, 7, 9, 11, 13, 15]
srcs = [torch.randint(0, 255, (H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(4)]
gd = torch.randint(0, 255, (H, W, 3), dtype=torch.uint8, device="cuda")
dst = torch.empty_like(srcs[0])


def taps(r):
    return sum(1 for y in range(-r, r + 1) for x in range(-r, r + 1) if x * x + y * y <= r * r)


for k in ks:
    b = _BilateralImpl(W, H, k)
    t0, i = time.perf_counter(), 0
    while time.perf_counter() - t0 < 1.0:
        b.joint_bilateral_filter(srcs[i % 4], gd, dst)
        i += 1
        if i % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    with vip.kernel_timing(64) as kt:
        for j in range(20):
            b.joint_bilateral_filter(srcs[j % 4], gd, dst)
    d = {n.split("(")[0]: round(1e3 * sum(v) / len(v), 2) for n, v in kt.durations().items()}
    us = sum(d.values())
    from oracle import oracle as o  # parity of this build on a ragged frame (test infrastructure)
    img = o.random_u8(121 * 203 * 3).reshape(121, 203, 3)
    g = o.random_u8(121 * 203 * 3, 200).reshape(121, 203, 3)
    out = torch.empty((121, 203, 3), dtype=torch.uint8, device="cuda")
    _BilateralImpl(203, 121, k).joint_bilateral_filter(torch.from_numpy(img).cuda(), torch.from_numpy(g).cuda(), out)
    torch.cuda.synchronize()
    ok = bool(np.array_equal(out.cpu().numpy(), o.joint_bilateral(img, g, k)))
    print(json.dumps({"k": k, "parity": ok, "us": round(us, 2), "gtaps_s": round(taps(k // 2) * W * H / us / 1e3, 1),
                      "kernels": list(d)}), flush=True)
