"""C4 (texture k=5, nitr=5, 4K) per frame with frames in flight on two streams, for
alternative library builds, each in its own process, run in the order given (pass the
builds interleaved for an A/B). One handle per stream, 12 rotating frames, 1 s clock
settle, then 400 frames between events.
usage: python scripts/experiments/texture_streams_ab.py variants/a.so variants/b.so ..."""
import json
import subprocess
import sys

CODE = r'''
import sys, json, time, torch
sys.path.insert(0, ".")
import various_image_processings_amd._lib as L
L.LIB_PATH = sys.argv[1]
from various_image_processings_amd.filters import _TextureImpl
W, H, S, N = 3840, 2160, 2, 400
srcs = [torch.randint(0, 255, (H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(12)]
dsts = [torch.empty_like(srcs[0]) for _ in range(12)]
streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(S - 1)]
tex = [_TextureImpl(W, H, 5, 5) for _ in range(S)]
raw = [s.cuda_stream for s in streams]
def frame(i):
    tex[i % S].execute(srcs[i % 12].data_ptr(), dsts[i % 12].data_ptr(), stream=raw[i % S])
t0 = time.perf_counter(); i = 0
while time.perf_counter() - t0 < 1.0:
    for _ in range(8):
        frame(i); i += 1
    torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(streams[0])
for s in streams[1:]:
    s.wait_event(e0)
for k in range(N):
    frame(i + k)
for s in streams[1:]:
    streams[0].wait_stream(s)
e1.record(streams[0]); torch.cuda.synchronize()
print(json.dumps({"ms_per_frame": round(e0.elapsed_time(e1) / N, 4)}))
'''
for so in sys.argv[1:]:
    r = subprocess.run([sys.executable, "-c", CODE, so], capture_output=True, text=True, timeout=300)
    print(so, r.stdout.strip() or r.stderr[-400:], flush=True)
