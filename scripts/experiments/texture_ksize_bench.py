"""Bilateral texture filter on a 4K frame for each texture ksize (the reference's default is 9,
C4 uses 5): the kernel-stamped duration of each launch of one iteration (the fused guide stage
and the joint bilateral of ksize 2k - 1), mean over 20 iterations after a 1 s clock settle.
usage: python scripts/experiments/texture_ksize_bench.py [--lib variants/x.so] [k ...]"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
args = sys.argv[1:]
if args[:1] == ["--lib"]:  # an alternative library build (scripts/build_*variant.sh)
    import various_image_processings_amd._lib as L
    L.LIB_PATH, args = args[1], args[2:]
import various_image_processings_amd as vip  # noqa: E402
from various_image_processings_amd.filters import _TextureImpl  # noqa: E402

W, H = 3840, 2160
ks = [int(a) for a in args] or [3, 4, 5, 7, 9, 11, 15, 24]
srcs = [torch.randint(0, 255, (H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(4)]
dst = torch.empty_like(srcs[0])
for k in ks:
    t = _TextureImpl(W, H, k, 1)
    t0 = time.perf_counter()
    i = 0
    while time.perf_counter() - t0 < 1.0:
        t.execute(srcs[i % 4], dst)
        i += 1
        if i % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    with vip.kernel_timing(64) as kt:
        for j in range(20):
            t.execute(srcs[j % 4], dst)
    d = {n.split("(")[0]: round(1e3 * sum(v) / len(v), 2) for n, v in kt.durations().items()}
    from oracle import oracle as o  # parity of this build on a ragged frame (test infrastructure)
    import numpy as np
    img = o.random_u8(121 * 203 * 3).reshape(121, 203, 3)
    out = torch.empty((121, 203, 3), dtype=torch.uint8, device="cuda")
    _TextureImpl(203, 121, k, 2).execute(torch.from_numpy(img).cuda(), out)
    torch.cuda.synchronize()
    ok = bool(np.array_equal(out.cpu().numpy(), o.texture(img, k, 2)))
    print(json.dumps({"k": k, "jbf_ksize": 2 * k - 1, "parity": ok, "us_per_launch": d}), flush=True)
