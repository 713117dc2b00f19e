"""Multi-frame slab launches (a rank's C2 / C3 slab at 2, 4, 8 GPUs: 2160 / N own rows +
two 7-row halos, 6 frames per launch, vip_*_run_rows_batch) on two streams, for
alternative library builds, each in its own process, in the order given (pass the builds
interleaved for an A/B). Per (filter, N, free_cus, streams): ms per frame over 600 frames
after a 1 s clock settle (one stream: launches back to back, none overlapping).
usage: python scripts/experiments/slab_batch_ab.py variants/a.so variants/b.so ..."""
import subprocess
import sys

CODE = r'''
import sys, json, time, torch
sys.path.insert(0, ".")
import various_image_processings_amd._lib as L
L.LIB_PATH = sys.argv[1]
from various_image_processings_amd.filters import _AdaptiveImpl, _BilateralImpl
W, r, B = 3840, 7, 6
res = {}
for kind, n, free, S in [("c2", 8, 8, 1), ("c2", 8, 8, 2), ("c2", 8, 16, 2), ("c2", 8, 0, 2), ("c2", 4, 32, 2),
                         ("c2", 2, 32, 2), ("c3", 8, 8, 1), ("c3", 8, 8, 2), ("c3", 4, 32, 2)]:
    own = 2160 // n; rows = own + 2 * r
    impl = [(_BilateralImpl if kind == "c2" else _AdaptiveImpl)(W, rows, 2 * r + 1) for _ in range(S)]
    srcs = [torch.randint(0, 255, (rows, W, 3), dtype=torch.uint8, device="cuda") for _ in range(12)]
    dsts = [torch.empty((own, W, 3), dtype=torch.uint8, device="cuda") for _ in range(12)]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(S - 1)]
    def group(i):
        fs = [(i * B + j) % 12 for j in range(B)]
        impl[i % S].run_rows_batch([srcs[f].data_ptr() for f in fs], [dsts[f].data_ptr() for f in fs], own, r, 0,
                                   rows, free_cus=free, stream=streams[i % S].cuda_stream)
    t0 = time.perf_counter(); i = 0
    while time.perf_counter() - t0 < 1.0:
        for _ in range(8):
            group(i); i += 1
        torch.cuda.synchronize()
    G = 100
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(streams[0])
    for s in streams[1:]:
        s.wait_event(e0)
    for k in range(G):
        group(i + k)
    for s in streams[1:]:
        streams[0].wait_stream(s)
    e1.record(streams[0]); torch.cuda.synchronize()
    res[f"{kind}_n{n}_free{free}_s{S}"] = round(e0.elapsed_time(e1) / (G * B), 5)
print(json.dumps(res))
'''
for so in sys.argv[1:]:
    r = subprocess.run([sys.executable, "-c", CODE, so], capture_output=True, text=True, timeout=300)
    print(so, r.stdout.strip() or r.stderr[-600:], flush=True)
