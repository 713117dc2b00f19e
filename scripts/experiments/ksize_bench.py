"""Time the large-ksize paths on a 4K frame (runtime-radius kernel, texture k=24), and
the runtime-radius kernel against the templated one at r=7 and r=15.
Prints one JSON line: per-launch microseconds, Mpx/s and G in-disc taps/s."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import various_image_processings_amd as vip  # noqa: E402
from various_image_processings_amd.filters import _AdaptiveImpl, _BilateralImpl, _TextureImpl  # noqa: E402

W, H = 3840, 2160
torch.cuda.set_device(0)
srcs = [torch.randint(0, 255, (H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(4)]
dst = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
guide = srcs[3]


def disc_taps(k):
    r = k // 2
    return sum(1 for y in range(-r, r + 1) for x in range(-r, r + 1) if x * x + y * y <= r * r)


def timed(f, n, settle_s=0.5):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < settle_s:
        f(srcs[0], dst)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(n):
        f(srcs[i % 3], dst)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


res = {}
cases = []
for k in (33, 65):
    b = _BilateralImpl(W, H, k)
    cases.append((f"bilateral_k{k}", b.bilateral_filter, disc_taps(k), 5))
j = _BilateralImpl(W, H, 47)
cases.append(("joint_k47", lambda s, d: j.joint_bilateral_filter(s, guide, d), disc_taps(47), 5))
a = _AdaptiveImpl(W, H, 63)
cases.append(("adaptive_k63", a.execute, disc_taps(63), 5))
t = _TextureImpl(W, H, 24, 1)
cases.append(("texture_k24_nitr1", t.execute, disc_taps(47), 5))
for name, f, taps, n in cases:
    us = timed(f, n)
    res[name] = {"us": round(us, 1), "mpx_s": round(W * H / us, 1), "gtaps_s": round(W * H * taps / us / 1e3, 1)}
    print(name, res[name], flush=True)
# runtime-radius kernel vs templated at radii both can run
for k in (15, 31):
    b = _BilateralImpl(W, H, k)
    ad = _AdaptiveImpl(W, H, k)
    for path in (vip.VIP_PATH_AUTO, vip.VIP_PATH_RUNTIME):
        vip.set_stencil_path(path)
        tag = "templated" if path == vip.VIP_PATH_AUTO else "runtime"
        for name, f in ((f"bilateral_k{k}_{tag}", b.bilateral_filter), (f"adaptive_k{k}_{tag}", ad.execute)):
            us = timed(f, 20 if k == 15 else 5)
            res[name] = {"us": round(us, 1), "gtaps_s": round(W * H * disc_taps(k) / us / 1e3, 1)}
            print(name, res[name], flush=True)
    vip.set_stencil_path(vip.VIP_PATH_AUTO)
print(json.dumps(res))
