"""Bit-exact check of an alternative libvip build against the oracle on small frames.
usage: python scripts/variant_parity.py variants/<name>.so"""
import sys

sys.path.insert(0, ".")
import various_image_processings_amd._lib as L

L.LIB_PATH = sys.argv[1]
import numpy as np
import torch

import various_image_processings_amd as vip
from oracle import oracle as o

img = o.random_image(389, 277)
guide = o.random_u8(389 * 277 * 3)[::-1].copy().reshape(277, 389, 3)
d, dg = torch.from_numpy(img).cuda(), torch.from_numpy(guide).cuda()
out = torch.empty_like(d)
ok = {}
for k in (9, 15):
    vip.CudaBilateralFilter(389, 277, k).bilateral_filter(d, out)
    ok[f"bilateral{k}"] = np.array_equal(out.cpu().numpy(), o.bilateral(img, k))
    vip.CudaBilateralFilter(389, 277, k).joint_bilateral_filter(d, dg, out)
    ok[f"joint{k}"] = np.array_equal(out.cpu().numpy(), o.joint_bilateral(img, guide, k))
    vip.CudaAdaptiveBilateralFilter(389, 277, k).execute(d, out)
    ok[f"adaptive{k}"] = np.array_equal(out.cpu().numpy(), o.adaptive(img, k))
vip.CudaBilateralTextureFilter(389, 277, 5, 2).execute(d, out)
ok["texture5"] = np.array_equal(out.cpu().numpy(), o.texture(img, 5, 2))
print(sys.argv[1], "parity", ok, flush=True)
sys.exit(0 if all(ok.values()) else 1)
