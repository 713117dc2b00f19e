"""C4 (texture k=5 nitr=5, 4K) per frame: direct launches vs one HIP graph per frame
(torch.cuda.CUDAGraph capturing the library's 10 launches on the capture stream), with 1
and 2 frames in flight. Also C2 (one launch) for reference. Outputs compared."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from various_image_processings_amd.filters import _BilateralImpl, _TextureImpl  # noqa: E402

torch.cuda.set_device(0)
W, H = 3840, 2160
srcs = [torch.randint(0, 255, (H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(4)]
dsts = [torch.empty((H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(4)]
res = {}


def timeit(frame, n=200):
    t0 = time.perf_counter()
    i = 0
    while time.perf_counter() - t0 < 1.0:
        for _ in range(4):
            frame(i)
            i += 1
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(n):
        frame(i + j)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


for name, mk in (("c4", lambda: _TextureImpl(W, H, 5, 5)), ("c2", lambda: _BilateralImpl(W, H, 15))):
    for S in (1, 2):
        streams = [torch.cuda.Stream() for _ in range(S)]
        hs = [mk() for _ in range(S)]
        run = (lambda h, a, b, s: h.execute(a, b, stream=s)) if name == "c4" else \
              (lambda h, a, b, s: h.bilateral_filter(a, b, stream=s))

        def direct(i):
            k = i % S
            run(hs[k], srcs[i % 4].data_ptr(), dsts[i % 4].data_ptr(), streams[k].cuda_stream)
        res[f"{name}_S{S}_direct_ms"] = round(timeit(direct), 4)
        # one graph per (stream, buffer): each captured on its stream
        graphs = {}
        for k in range(S):
            for b in range(4):
                if b % S != k:
                    continue
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=streams[k]):
                    run(hs[k], srcs[b].data_ptr(), dsts[b].data_ptr(), streams[k].cuda_stream)
                graphs[(k, b)] = g

        def replay(i):
            k = i % S
            b = i % 4
            if b % S != k:
                b = k
            with torch.cuda.stream(streams[k]):
                graphs[(k, b)].replay()
        res[f"{name}_S{S}_graph_ms"] = round(timeit(replay), 4)
        print(name, S, res, flush=True)
# outputs equal
t = _TextureImpl(W, H, 5, 5)
t.execute(srcs[0], dsts[0])
torch.cuda.synchronize()
want = dsts[0].clone()
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
with torch.cuda.graph(g, stream=s):
    t.execute(srcs[0].data_ptr(), dsts[1].data_ptr(), stream=s.cuda_stream)
g.replay()
torch.cuda.synchronize()
res["graph_output_equal"] = bool(torch.equal(want, dsts[1]))
print(json.dumps(res))
