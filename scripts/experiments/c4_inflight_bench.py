"""C4 (texture k=5 nitr=5, 4K) per-frame time with S frames in flight on S streams, for
alternative library builds (each in its own subprocess).
usage: python scripts/experiments/c4_inflight_bench.py lib1.so [lib2.so ...]"""
import os
import subprocess
import sys

CODE = r'''
import sys, json, time, torch
sys.path.insert(0, ".")
import various_image_processings_amd._lib as L
L.LIB_PATH = sys.argv[1]
from various_image_processings_amd.filters import _TextureImpl
torch.cuda.set_device(0)
W, H = 3840, 2160
srcs = [torch.randint(0, 255, (H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(6)]
dsts = [torch.empty((H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(6)]
res = {}
for S in (1, 2, 3):
    streams = [torch.cuda.Stream() for _ in range(S)]
    texs = [_TextureImpl(W, H, 5, 5) for _ in range(S)]
    def frame(i):
        h = i % S
        texs[h].execute(srcs[i % 6].data_ptr(), dsts[i % 6].data_ptr(), stream=streams[h].cuda_stream)
    t0 = time.perf_counter(); i = 0
    while time.perf_counter() - t0 < 1.0:
        for _ in range(6): frame(i); i += 1
        torch.cuda.synchronize()
    torch.cuda.synchronize()
    n = 240
    t0 = time.perf_counter()
    for j in range(n): frame(i + j)
    torch.cuda.synchronize()
    res[f"S{S}_ms_per_frame"] = round((time.perf_counter() - t0) / n * 1e3, 4)
print(json.dumps(res))
'''
for so in sys.argv[1:]:
    r = subprocess.run([sys.executable, "-c", CODE, so], capture_output=True, text=True, timeout=300)
    print(os.path.basename(so), r.stdout.strip() or r.stderr[-800:], flush=True)
