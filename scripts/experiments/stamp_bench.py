"""Diagnostic: run the stamped bilateral build once on a 4K frame and summarise
per-tile wave timelines (compute span, barrier wait). usage: stamp_bench.py variants/stamps.so"""
import ctypes, sys, json
import numpy as np
sys.path.insert(0, ".")
import various_image_processings_amd._lib as L
L.LIB_PATH = sys.argv[1]
import torch
from various_image_processings_amd.filters import _BilateralImpl
W, H = 3840, 2160
src = torch.randint(0, 255, (H, W, 3), dtype=torch.uint8, device="cuda")
dst = torch.empty_like(src)
f = _BilateralImpl(W, H, 15)
for _ in range(3):
    f.bilateral_filter(src, dst)
torch.cuda.synchronize()
buf = np.zeros(256 * 16 * 8 * 3, np.uint64)
lib = L.lib()
lib.vip_debug_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert lib.vip_debug_read_stamps(buf.ctypes.data, buf.nbytes) == 0
s = buf.reshape(256, 16, 8, 3).astype(np.int64)
res = {}
t0 = s[:, :, :, 0]; t1 = s[:, :, :, 1]; t2 = s[:, :, :, 2]
valid = (t0 > 0) & (t1 > t0)
comp = np.where(valid, t1 - t0, 0)
for it in range(4):
    v = valid[:, :, it]
    if not v.any():
        continue
    c = comp[:, :, it][v]
    last = np.max(np.where(v, t1[:, :, it], 0), axis=1)
    first = np.min(np.where(v, t1[:, :, it], 2**62), axis=1)
    spread = (last - first)[v.any(axis=1)]
    has2 = v & (t2[:, :, it] > t1[:, :, it])
    bar = (t2[:, :, it] - t1[:, :, it])[has2] if has2.any() else np.array([0])
    res[f"tile{it}"] = dict(compute_med=int(np.median(c)), compute_min=int(c.min()), compute_max=int(c.max()),
                            finish_spread_med=int(np.median(spread)), barrier_wait_med=int(np.median(bar)),
                            barrier_wait_max=int(bar.max()))
# whole-kernel span per block
start = np.min(np.where(t0 > 0, t0, 2**62), axis=(1, 2)); end = np.max(np.where(t1 > 0, t1, 0), axis=(1, 2))
res["block_span_med"] = int(np.median(end - start)); res["global_span"] = int(end.max() - start.min())
# per-wave-slot (wave index within block) mean compute of tile 0: priority effect
res["tile0_compute_by_wave"] = [int(x) for x in comp[:, :, 0].mean(axis=0)]
print(json.dumps(res, indent=1))

# in-kernel clock and residency (wave 0 of each block: entry/exit shader clock and
# 100 MHz real time), against the event-timed launch
if hasattr(lib, "vip_debug_read_rt"):
    rt = np.zeros(256 * 4, np.uint64)
    lib.vip_debug_read_rt.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); f.bilateral_filter(src, dst); e1.record(); torch.cuda.synchronize()
    assert lib.vip_debug_read_rt(rt.ctypes.data, rt.nbytes) == 0
    r = rt.reshape(256, 4).astype(np.int64)
    clk = (r[:, 2] - r[:, 0]) / np.maximum(r[:, 3] - r[:, 1], 1) * 0.1  # GHz
    ent, ext = (r[:, 1] - r[:, 1].min()) * 10, (r[:, 3] - r[:, 1].min()) * 10  # ns
    print(json.dumps(dict(event_us=round(e0.elapsed_time(e1) * 1e3, 1), clock_ghz_med=round(float(np.median(clk)), 3),
                          clock_ghz_min=round(float(clk.min()), 3), entry_spread_us=round(float(ent.max()) / 1e3, 2),
                          exit_first_us=round(float(ext.min()) / 1e3, 1), exit_last_us=round(float(ext.max()) / 1e3, 1),
                          block_span_med_us=round(float(np.median(ext - ent)) / 1e3, 1))))
    xcd = np.arange(256) % 8
    print(json.dumps(dict(exit_pct_us=[round(float(np.percentile(ext, q)) / 1e3, 1) for q in (0, 2, 5, 25, 50, 75, 95, 100)],
                          exit_med_by_xcd_us=[round(float(np.median(ext[xcd == x])) / 1e3, 1) for x in range(8)],
                          clock_by_xcd_ghz=[round(float(np.median(clk[xcd == x])), 3) for x in range(8)],
                          entry_by_xcd_us=[round(float(np.median(ent[xcd == x])) / 1e3, 2) for x in range(8)])))
