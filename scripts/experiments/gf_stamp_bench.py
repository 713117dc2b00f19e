"""Diagnostic: phase timeline of the fused texture guide stage (VIP_GF_STAMPS build).
Runs one 4K k=5 iteration, reads [workgroup][wave][8] shader-clock stamps (entry, arrival
at each of the 6 phase barriers, exit) and prints, per phase, the mean duration from the
previous barrier's last arrival to each wave's arrival (work) and to the last wave's
arrival (phase length, i.e. incl. the wait for the slowest wave).
usage: python scripts/experiments/gf_stamp_bench.py variants/<stamps>.so"""
import ctypes
import json
import sys

import numpy as np

sys.path.insert(0, ".")
import various_image_processings_amd._lib as L  # noqa: E402

L.LIB_PATH = sys.argv[1]
import torch  # noqa: E402

from various_image_processings_amd.filters import _TextureImpl  # noqa: E402

W, H = 3840, 2160
src = torch.randint(0, 255, (H, W, 3), dtype=torch.uint8, device="cuda")
dst = torch.empty_like(src)
f = _TextureImpl(W, H, 5, 1)
for _ in range(3):
    f.execute(src, dst)
torch.cuda.synchronize()
buf = np.zeros(4096 * 16 * 16, np.uint64)
lib = L.lib()
lib.vip_debug_read_gf_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert lib.vip_debug_read_gf_stamps(buf.ctypes.data, buf.nbytes) == 0
s = buf.reshape(4096, 16, 16).astype(np.int64)
valid = (s[:, 0, 0] > 0) & (s[:, 0, 7] > s[:, 0, 0])
s = s[valid]
names = ["xr load", "gradient+pass1", "MR store", "pass2", "BR/RR store", "guide", "store"]
res = {"workgroups": int(valid.sum())}
start = s[:, :, 0].min(axis=1)  # first wave's entry
prev = start
tot = (s[:, :, 7].max(axis=1) - start).mean()
for k in range(1, 8):
    arr = s[:, :, k]
    work = (arr - prev[:, None]).mean()
    length = (arr.max(axis=1) - prev).mean()
    res[names[k - 1]] = {"mean_wave_work": round(float(work)), "phase_length": round(float(length)),
                         "share": round(float(length / tot), 3)}
    prev = arr.max(axis=1)
res["tile_lifetime_cycles"] = round(float(tot))
# inside phases, per wave: XR loads issued (8) and gradients done (9)
res["xr issue (entry -> loads issued)"] = round(float((s[:, :, 8] - start[:, None]).mean()))
res["xr wait+unpack (issued -> barrier arrival)"] = round(float((s[:, :, 1] - s[:, :, 8]).mean()))
b1 = s[:, :, 1].max(axis=1)
res["gradients (barrier 1 -> done)"] = round(float((s[:, :, 9] - b1[:, None]).mean()))
res["pass 1 (gradients done -> barrier 2 arrival)"] = round(float((s[:, :, 2] - s[:, :, 9]).mean()))
# concurrency: how many workgroups overlap in time per CU is not visible here; the
# span of all stamps gives the kernel's clock count
res["kernel_span_cycles"] = int(s[:, :, 7].max() - s[:, :, 0].min())
print(json.dumps(res, indent=1))
