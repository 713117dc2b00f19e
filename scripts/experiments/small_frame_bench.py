"""Bilateral launch time per frame size for each tiling of the plain kernel
(VIP_BIL_WAVES=16|8|4 x VIP_BIL_WIDE=1 (128-px tiles) | 2 (256-px tiles), or the
library's own choice), one subprocess per setting (the knobs are read once per process). Every forced setting's output must equal the
auto setting's byte for byte (same arithmetic, different tiles).
usage: python scripts/experiments/small_frame_bench.py [out.json]"""
import json
import os
import subprocess
import sys

CODE = r'''
import sys, json, time, torch
sys.path.insert(0, ".")
from various_image_processings_amd.filters import _BilateralImpl
torch.cuda.set_device(0)
cases = [("c1_lenna_r5", 512, 512, 11), ("720p_r7", 1280, 720, 15), ("1080p_r7", 1920, 1080, 15),
         ("4k_r7", 3840, 2160, 15), ("720p_r3", 1280, 720, 7),
         # slabs of the 4K frame at 2 / 4 / 8 GPUs and a 7-row edge band (strong scaling)
         ("4k_slab1080_r7", 3840, 1080, 15), ("4k_slab540_r7", 3840, 540, 15), ("4k_slab270_r7", 3840, 270, 15),
         ("4k_band7_r7", 3840, 7, 15)]
res, sums = {}, {}
g = torch.Generator(device="cuda"); g.manual_seed(7)
for name, W, H, k in cases:
    srcs = [torch.randint(0, 255, (H, W, 3), dtype=torch.uint8, device="cuda", generator=g) for _ in range(6)]
    dst = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
    f = _BilateralImpl(W, H, k).bilateral_filter
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.7:
        for i in range(16): f(srcs[i % 6], dst)
        torch.cuda.synchronize()
    n = 400 if W * H < 4e6 else 100
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(n): f(srcs[i % 6], dst)
    e1.record(); torch.cuda.synchronize()
    res[name + "_us"] = round(e0.elapsed_time(e1) / n * 1e3, 2)
    f(srcs[0], dst); torch.cuda.synchronize()
    sums[name] = int((dst.to(torch.int64) * torch.arange(1, dst.numel() + 1, device="cuda").view(dst.shape) % 1000003).sum().item())
print(json.dumps({"us": res, "sums": sums}))
'''
out = {}
for w in ["auto", "16", "8", "4", "16w", "8w", "4w"]:
    env = dict(os.environ)
    env.pop("VIP_BIL_WAVES", None)
    env.pop("VIP_BIL_WIDE", None)
    if w != "auto":
        env["VIP_BIL_WAVES"] = w.rstrip("w")
        env["VIP_BIL_WIDE"] = "2" if w.endswith("w") else "1"
    r = subprocess.run([sys.executable, "-c", CODE], capture_output=True, text=True, timeout=240, env=env)
    if r.returncode != 0:
        print(w, r.stderr[-800:], flush=True)
        sys.exit(r.returncode)
    out[w] = json.loads(r.stdout.strip().splitlines()[-1])
    print(w, json.dumps(out[w]["us"]), flush=True)
ok = all(out[w]["sums"] == out["auto"]["sums"] for w in out)
print("outputs equal across wave counts:", ok)
if len(sys.argv) > 1:
    with open(sys.argv[1], "w") as fh:
        json.dump({"equal": ok, **out}, fh, indent=1)
sys.exit(0 if ok else 1)
