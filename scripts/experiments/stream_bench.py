#!/usr/bin/env python3
"""Frames in flight on S HIP streams vs one stream (steady clocks, 4K frames).

For each config and S, frames i = 0..K-1 go round-robin to S streams (one filter
handle per stream: a texture handle owns scratch frames), after a 1 s clock settle;
the time per frame is the wall time of the K frames / K. Prints one line per (config,
S). Diagnostic for bench.py --streams."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from various_image_processings_amd.filters import _AdaptiveImpl, _BilateralImpl, _TextureImpl  # noqa: E402

W, H, NBUF = 3840, 2160, 12


def make(kind):
    if kind == "c2":
        h = _BilateralImpl(W, H, 15)
        return h, lambda s, d, st: h.bilateral_filter(s, d, stream=st)
    if kind == "c3":
        h = _AdaptiveImpl(W, H, 15)
        return h, lambda s, d, st: h.execute(s, d, stream=st)
    h = _TextureImpl(W, H, 5, 5)
    return h, lambda s, d, st: h.execute(s, d, stream=st)


def run(kind, nstreams, steps):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    srcs = [torch.randint(0, 255, (H, W, 3), dtype=torch.uint8, device=dev, generator=g) for _ in range(NBUF)]
    dsts = [torch.empty_like(srcs[0]) for _ in range(NBUF)]
    streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
    hs = [make(kind) for _ in range(nstreams)]

    def frame(i):
        k = i % nstreams
        hs[k][1](srcs[i % NBUF], dsts[i % NBUF], streams[k])

    t0, i = time.perf_counter(), 0
    while time.perf_counter() - t0 < 1.0:
        for _ in range(8):
            frame(i)
            i += 1
        torch.cuda.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(steps):
        frame(j)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"{kind} streams={nstreams} steps={steps} ms/frame={dt * 1e3:.4f} Mpx/s={W * H / dt / 1e6:.0f}", flush=True)


if __name__ == "__main__":
    cfgs = sys.argv[1:] or ["c2", "c3", "c4"]
    steps = {"c2": 2000, "c3": 1000, "c4": 500}
    for c in cfgs:
        for s in (1, 2, 3, 1):
            run(c, s, steps[c])
