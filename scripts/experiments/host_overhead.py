"""Host time per launch of the C1 bilateral (512x512, ksize 11) through each Python
layer, without synchronising inside the loop (the queue absorbs the launches): the
bench path (ShardedBilateral.filter), the handle's run_rows, and a bare ctypes call
of vip_bilateral_run_rows with pre-converted arguments. usage: python scripts/experiments/host_overhead.py"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import various_image_processings_amd as vip  # noqa: E402
from various_image_processings_amd.sharded import ShardedBilateral  # noqa: E402

torch.cuda.set_device(0)
W = H = 512
srcs = [torch.randint(0, 255, (H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(4)]
dst = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
sb = ShardedBilateral(W, H, 11, 0, 1)
s = torch.cuda.current_stream().cuda_stream
sp = [t.data_ptr() for t in srcs]
dp = dst.data_ptr()
lo, hi = sb.geo.clamp_range()
fn = vip.lib().vip_bilateral_run_rows
h = sb.impl._h
p = W * 3


def t(label, f, n=4000):
    for i in range(200):
        f(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        f(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return label, round((t1 - t0) / n * 1e6, 2), round((t2 - t0) / n * 1e6, 2)


small = [t("bare ctypes call, 300 launches", lambda i: fn(h, sp[i & 3], p, None, p, dp, p, H, 0, lo, hi, s), n=300),
         t("ctypes call of vip_abi_version (no HIP work)", lambda i: vip.lib().vip_abi_version(), n=300),
         t("torch fill_ launch, 300", lambda i: dst.fill_(i & 7), n=300)]
res = small + [t("bench path (ShardedBilateral.filter)", lambda i: sb.filter(sp[i & 3], dp, stream=s, exchange=False)),
       t("handle run_rows", lambda i: sb.impl.run_rows(sp[i & 3], dp, H, 0, lo, hi, stream=s)),
       t("bare ctypes call", lambda i: fn(h, sp[i & 3], p, None, p, dp, p, H, 0, lo, hi, s))]
print(json.dumps([{"path": a, "host_us_per_launch": b, "wall_us_per_launch": c} for a, b, c in res], indent=1))
