"""C4 guide-stage A/B: alternative library builds, each in its own process, in the order
given (pass them interleaved). Per build: bit-exact texture outputs against the oracle on a
few ragged frames, then on a 4K C4 frame (k = 5, nitr = 5, 12 rotating inputs, 1 s clock
settle) the kernel durations of the guide stage and the JBF on one stream
(vip_kernel_timing: kernel-stamped events), the one-stream ms per frame, and the ms per frame
with two frames in flight (two streams, one handle each).
usage: python scripts/experiments/guide_stage_ab.py variants/a.so variants/b.so ..."""
import subprocess
import sys

CODE = r'''
import sys, json, time, torch
import numpy as np
sys.path.insert(0, ".")
import various_image_processings_amd._lib as L
L.LIB_PATH = sys.argv[1]
import various_image_processings_amd as vip
from various_image_processings_amd.filters import _TextureImpl
from oracle import oracle as o
res = {}
ok = True
for (h, w, k, n) in ((277, 389, 5, 2), (121, 203, 4, 2), (7, 130, 5, 1), (300, 257, 5, 1)):
    img = o.random_u8(h * w * 3).reshape(h, w, 3)
    d = torch.from_numpy(img).cuda(); out = torch.empty_like(d)
    _TextureImpl(w, h, k, n).execute(d, out); torch.cuda.synchronize()
    ok = ok and np.array_equal(out.cpu().numpy(), o.texture(img, k, n))
res["parity"] = ok
W, H, S = 3840, 2160, 2
srcs = [torch.randint(0, 255, (H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(12)]
dsts = [torch.empty_like(srcs[0]) for _ in range(12)]
streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(S - 1)]
tex = [_TextureImpl(W, H, 5, 5) for _ in range(S)]
raw = [s.cuda_stream for s in streams]
def frame(i, h=None):
    h = i % S if h is None else h
    tex[h].execute(srcs[i % 12].data_ptr(), dsts[i % 12].data_ptr(), stream=raw[h])
t0 = time.perf_counter(); i = 0
while time.perf_counter() - t0 < 1.0:
    for _ in range(8):
        frame(i); i += 1
    torch.cuda.synchronize()
def timed(n, one):
    global i
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(streams[0])
    for s in streams[1:]:
        s.wait_event(e0)
    for k in range(n):
        frame(i + k, 0 if one else None)
    i += n
    for s in streams[1:]:
        streams[0].wait_stream(s)
    e1.record(streams[0]); torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n, 4)
res["two_stream_ms"] = timed(400, False)
with vip.kernel_timing(1000) as kt:
    res["one_stream_ms"] = timed(100, True)
res["kernels_us"] = {n.split("<")[0].split("::")[-1] + "<" + n.split("<", 1)[1][:12]: round(1e3 * sum(v) / len(v), 2)
                     for n, v in kt.durations().items()}
res["two_stream_ms_2"] = timed(400, False)
print(json.dumps(res))
'''
for so in sys.argv[1:]:
    r = subprocess.run([sys.executable, "-c", CODE, so], capture_output=True, text=True, timeout=300)
    print(so, r.stdout.strip() or r.stderr[-600:], flush=True)
    if r.returncode != 0:  # a fault or abort ends the run: nothing more on the GPU
        sys.exit(r.returncode if r.returncode > 0 else 1)
