"""Time bilateral (and adaptive) r=7 on a 4K frame with an alternative libvip build.
usage: python scripts/variant_bench.py variants/<name>.so [...]  (each in a subprocess)"""
import json
import os
import subprocess
import sys

CODE = r'''
import sys, json, torch, ctypes
sys.path.insert(0, ".")
import various_image_processings_amd._lib as L
L.LIB_PATH = sys.argv[1]
_h = ctypes.CDLL(sys.argv[1])  # an older build lacks newer entry points: bind only what it has
for _n in [n for n in L.SIGNATURES if not hasattr(_h, n)]:
    del L.SIGNATURES[_n]
from various_image_processings_amd.filters import _BilateralImpl, _AdaptiveImpl, _TextureImpl
torch.cuda.set_device(0)
W, H = 3840, 2160
srcs = [torch.randint(0, 255, (H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(6)]
dst = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
res = {}
guide = srcs[5]
cases = [("bilateral", _BilateralImpl(W, H, 15).bilateral_filter),
         ("adaptive", _AdaptiveImpl(W, H, 15).execute)]
j9, j15 = _BilateralImpl(W, H, 9), _BilateralImpl(W, H, 15)
jt = _BilateralImpl(W, H, 9, 4.0, 1.73205080757)  # the texture filter's JBF at k = 5
cases += [("joint_r4", lambda s, d: j9.joint_bilateral_filter(s, guide, d)),
          ("joint_r4_texture_sigmas", lambda s, d: jt.joint_bilateral_filter(s, guide, d)),
          ("joint_r7", lambda s, d: j15.joint_bilateral_filter(s, guide, d)),
          ("texture_k5_nitr1", _TextureImpl(W, H, 5, 1).execute),
          ("texture_k5_nitr5", _TextureImpl(W, H, 5, 5).execute)]
def fused(nitr):  # vip_texture_set_mode(FUSED): guide + JBF in one launch per iteration
    t = _TextureImpl(W, H, 5, nitr)
    t.set_mode(_TextureImpl.FUSED)
    return t.execute
try:
    cases += [("texture_k5_nitr1_fused", fused(1)), ("texture_k5_nitr5_fused", fused(5))]
except Exception:  # an older library without the mode
    pass
if "--r15" in sys.argv:  # one 2048-row slab of the C5 frame (16384 wide, ksize 31)
    s15 = [torch.randint(0, 255, (2048 + 30, 16384, 3), dtype=torch.uint8, device="cuda") for _ in range(2)]
    d15 = torch.empty((2048 + 30, 16384, 3), dtype=torch.uint8, device="cuda")
    b31 = _BilateralImpl(16384, 2048 + 30, 31)
    cases += [("bilateral_r15_slab", lambda s, d: b31.bilateral_filter(s15[0], d15))]
import time
only = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--only=")]
for name, f in cases:
    if only and not any(name.startswith(o) for o in only):
        continue
    # clock settle: 1 s of back-to-back launches (MI355X clocks ramp under sustained load)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        for i in range(8): f(srcs[i % 6], dst)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 100
    e0.record()
    for i in range(n): f(srcs[i % 6], dst)
    e1.record(); torch.cuda.synchronize()
    res[name + "_us"] = round(e0.elapsed_time(e1) / n * 1e3, 1)
print(json.dumps(res))
'''
extra = [a for a in sys.argv[1:] if a.startswith("--")]
for so in [a for a in sys.argv[1:] if not a.startswith("--")]:
    r = subprocess.run([sys.executable, "-c", CODE, so] + extra, capture_output=True, text=True, timeout=300)
    print(os.path.basename(so), r.stdout.strip() or r.stderr[-500:], flush=True)
