"""Graph mode of the native shard inside a torch process (whose RCCL and HIP runtime are
torch's own copies, which libvip_shard.so's symbols bind to): loopback shards, one per
stream, frames replayed from captured graphs against their direct runs. Run in a child
process of its own (a crash here ends only this probe).
usage: python scripts/experiments/graph_probe.py [split] [trace] [sysrccl]"""
import faulthandler
import sys

sys.path.insert(0, ".")
faulthandler.enable()
if "trace" in sys.argv:  # native backtrace of a crash (microbench/segv_trace.c)
    import ctypes
    ctypes.CDLL("microbench/libsegv_trace.so").segv_trace_install()
if "sysrccl" in sys.argv:  # the system HIP 7.2 + RCCL 2.27.7 loaded before torch's own copies
    import ctypes
    for lib in ("/opt/rocm/lib/libamdhip64.so.7", "/opt/rocm/lib/librccl.so.1"):
        ctypes.CDLL(lib, mode=ctypes.RTLD_GLOBAL)
import torch  # noqa: E402

from various_image_processings_amd.sharded import NativeShard  # noqa: E402

split = "split" in sys.argv[1:]
torch.cuda.set_device(0)
w, own, n = 3840, 270, 8
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
shards = [NativeShard(w, n * own, 15, n // 2, n, None, loopback=True) for _ in streams]
g = torch.Generator(device="cuda")
g.manual_seed(1)
slabs = [torch.randint(0, 255, (own + 14, w, 3), dtype=torch.uint8, device="cuda", generator=g) for _ in range(4)]
ref = [torch.empty((own, w, 3), dtype=torch.uint8, device="cuda") for _ in slabs]
out = [torch.empty_like(x) for x in ref]
launch = [x.launcher() for x in shards]
for x in shards:
    x.set_split(split)


def rnd(dst):
    for i in range(len(slabs)):
        h = i % 2
        launch[h](slabs[i].data_ptr(), dst[i].data_ptr(), streams[h].cuda_stream)


rnd(ref)
torch.cuda.synchronize()
print("direct run done", flush=True)
for x in shards:
    x.set_graph(True)
for r in range(3):
    for o in out:
        o.fill_(3)
    torch.cuda.synchronize()
    rnd(out)
    torch.cuda.synchronize()
    print(f"graph round {r}: equal = {all(torch.equal(a, b) for a, b in zip(out, ref))}, "
          f"graphs = {[x.graph_count() for x in shards]}", flush=True)
