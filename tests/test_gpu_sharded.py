"""Row-sharded path on the GPU with the real HIP kernels.

Two ranks share the one GPU of the test box (gloo moves the halo rows through host
memory; with one process per GPU the same exchange_halo calls run over RCCL/xGMI).
Each rank filters its slab with ShardedBilateral / ShardedTexture -- the HIP row-band
kernels with the clamp range of its position in the frame -- and the concatenated
slabs must equal the oracle's single-frame result bit for bit.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, width, height, ksize, kind, nitr, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    from oracle import oracle as o
    from various_image_processings_amd.sharded import ShardedBilateral, ShardedTexture

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    frame = o.random_image(width, height)
    if kind == "texture":
        sh = ShardedTexture(width, height, ksize, nitr, rank, world)
    else:
        sh = ShardedBilateral(width, height, ksize, rank, world, adaptive=kind == "adaptive")
    g = sh.geo
    b, e = g.rows
    slab = torch.zeros((g.slab_rows, width, 3), dtype=torch.uint8, device="cuda")
    slab[g.radius:g.radius + g.own] = torch.from_numpy(frame[b:e]).cuda()  # only own rows are local
    out = torch.empty((g.own, width, 3), dtype=torch.uint8, device="cuda")
    sh.filter(slab, out)  # exchange_halo + the HIP row-band kernel(s)
    torch.cuda.synchronize()
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), out.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,width,height,ksize,kind,nitr", [
    (2, 301, 173, 15, "bilateral", 0),
    (3, 257, 140, 31, "bilateral", 0),
    (2, 190, 121, 15, "adaptive", 0),
    (2, 211, 150, 5, "texture", 3),
    (8, 613, 400, 31, "bilateral", 0),  # C5's 8-way split (r=15) with a real gloo exchange
])
def test_sharded_hip_kernels_match_full_frame(tmp_path, world, width, height, ksize, kind, nitr):
    import torch.multiprocessing as mp
    from oracle import oracle as o
    mp.start_processes(_worker, args=(world, _free_port(), width, height, ksize, kind, nitr, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    got = np.concatenate([np.load(tmp_path / f"rank{i}.npy") for i in range(world)], axis=0)
    frame = o.random_image(width, height)
    if kind == "texture":
        want = o.texture(frame, ksize, nitr)
    else:
        want = (o.adaptive if kind == "adaptive" else o.bilateral)(frame, ksize)
    assert np.array_equal(got, want)
