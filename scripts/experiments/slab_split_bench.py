"""Per-rank compute of C2 strong scaling on one GPU: a (3840 x (2160/N + 14)) slab of the
4K frame filtered (a) as one launch over its own rows, (b) split -- interior rows, then
the two 7-row edge bands on the same stream, (c) split like vip_shard_run -- the edge
bands on a side stream concurrent with the interior -- with 1 and 2 frames in flight.
Excludes the exchange. Prints one JSON line per N."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from various_image_processings_amd.filters import _BilateralImpl  # noqa: E402
from various_image_processings_amd.sharded import SlabGeometry, split_bands  # noqa: E402

W, H, K = 3840, 2160, 15
torch.cuda.set_device(0)
for n in (1, 2, 4, 8):
    geo = SlabGeometry(W, H, K // 2, 1 if n > 1 else 0, n)  # an interior rank: halos on both sides
    r, own = geo.radius, geo.own
    impl = _BilateralImpl(W, geo.slab_rows, K)
    lo, hi = geo.clamp_range()
    slabs = [torch.randint(0, 255, (geo.slab_rows, W, 3), dtype=torch.uint8, device="cuda") for _ in range(4)]
    outs = [torch.empty((own, W, 3), dtype=torch.uint8, device="cuda") for _ in range(4)]
    (i0, ni), edges = split_bands(geo)
    res = {"n": n, "own_rows": own}
    for mode in ("full", "split", "split_side"):
        for S in (1, 2):
            streams = [torch.cuda.Stream() for _ in range(S)]
            sides = [torch.cuda.Stream() for _ in range(S)]  # vip_shard's communication streams

            def frame(i):
                s = streams[i % S]
                sl, o = slabs[i % 4], outs[i % 4]
                if mode == "full":
                    impl.run_rows(sl, o, own, r, lo, hi, stream=s)
                elif mode == "split":  # edges after the interior, one stream
                    impl.run_rows(sl, o[i0:i0 + ni], ni, r + i0, lo, hi, stream=s)
                    for e0, ne in edges:
                        impl.run_rows(sl, o[e0:e0 + ne], ne, r + e0, lo, hi, stream=s)
                else:  # vip_shard_run: edges on the side stream, concurrent with the interior
                    c = sides[i % S]
                    c.wait_stream(s)
                    for e0, ne in edges:
                        impl.run_rows(sl, o[e0:e0 + ne], ne, r + e0, lo, hi, stream=c)
                    impl.run_rows(sl, o[i0:i0 + ni], ni, r + i0, lo, hi, stream=s)
                    s.wait_stream(c)
            t0 = time.perf_counter()
            i = 0
            while time.perf_counter() - t0 < 0.7:
                for _ in range(8):
                    frame(i)
                    i += 1
                torch.cuda.synchronize()
            m = 400
            t0 = time.perf_counter()
            for j in range(m):
                frame(i + j)
            torch.cuda.synchronize()
            res[f"{mode}_S{S}_us"] = round((time.perf_counter() - t0) / m * 1e6, 1)
    print(json.dumps(res), flush=True)
