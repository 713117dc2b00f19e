"""Row-sharded multi-process path on CPU (gloo, world_size 2, 3 and 8).

Each rank owns a row slab plus r-row halos; exchange_halo() fills the halos from
the neighbouring ranks with point-to-point send/recv (the same calls run over
RCCL/xGMI with the nccl backend on GPUs). The per-slab filter here is the
oracle's row-band function (test infrastructure standing in for the HIP kernel,
which needs a GPU); the test checks that sharding + halo exchange + the clamp
range reproduce the single-frame result exactly.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, width, height, ksize, kind, nitr, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import oracle as o
    from various_image_processings_amd.sharded import SlabGeometry, exchange_halo, texture_halo_rows

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frame = o.random_image(width, height)
    halo = nitr * texture_halo_rows(ksize) if kind == "texture" else ksize // 2
    geo = SlabGeometry(width, height, halo, rank, world)
    b, e = geo.rows
    r = geo.radius
    slab = torch.zeros((geo.slab_rows, width, 3), dtype=torch.uint8)
    slab[r:r + geo.own] = torch.from_numpy(frame[b:e])  # only own rows are local
    exchange_halo(slab, geo)
    lo, hi = geo.clamp_range()
    s = slab.numpy()
    # halo rows must equal the neighbours' edge rows
    if geo.has_above:
        assert np.array_equal(s[:r], frame[b - r:b])
    if geo.has_below:
        assert np.array_equal(s[r + geo.own:], frame[e:e + r])
    # the band filter over the clamp range == the frame filter's rows
    view = s[lo:hi]
    if kind == "texture":  # the slab filtered as a frame: its own rows are exact given the halo
        band = o.texture(np.ascontiguousarray(view), ksize, nitr)[r - lo:r - lo + geo.own]
    else:
        fn = o.adaptive if kind == "adaptive" else o.bilateral
        band = fn(np.ascontiguousarray(view), ksize)[r - lo:r - lo + geo.own]
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), band)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,height,ksize,kind,nitr", [(2, 37, 9, "bilateral", 0), (3, 50, 15, "bilateral", 0),
                                                          (2, 31, 31, "bilateral", 0),  # uneven 16/15-row shards, r=15
                                                          (2, 41, 7, "adaptive", 0), (2, 70, 5, "texture", 3),
                                                          (3, 90, 3, "texture", 4),
                                                          (8, 83, 9, "bilateral", 0),  # the driver's N = 8, ragged
                                                          (8, 371, 5, "texture", 5)])  # C4 k, nitr at N = 8: 46-row shards, 45-row halo
def test_row_sharded_halo_exchange_matches_full_frame(tmp_path, world, height, ksize, kind, nitr):
    """Texture: one exchange of nitr * texture_halo_rows(k) rows per frame
    (ShardedTexture's ghost-zone scheme) makes each slab's own rows exact."""
    from oracle import oracle as o
    width = 29
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, width, height, ksize, kind, nitr, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    got = np.concatenate([np.load(tmp_path / f"rank{i}.npy") for i in range(world)], axis=0)
    frame = o.random_image(width, height)
    if kind == "texture":
        want = o.texture(frame, ksize, nitr)
    else:
        want = (o.adaptive if kind == "adaptive" else o.bilateral)(frame, ksize)
    assert np.array_equal(got, want)


def test_shard_rows_partition():
    from various_image_processings_amd.sharded import SlabGeometry, shard_rows
    for h in (1, 7, 16384, 2161):
        for w in (1, 2, 3, 8):
            if w > h:
                continue
            spans = [shard_rows(h, w, i) for i in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == h
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(e - b for b, e in spans) - min(e - b for b, e in spans) <= 1
    g = SlabGeometry(3840, 16384, 15, 0, 8)
    assert g.clamp_range() == (15, 15 + 2048 + 15) and g.slab_rows == 2048 + 30
    g = SlabGeometry(3840, 16384, 15, 7, 8)
    assert g.clamp_range() == (0, 15 + 2048)


def test_thin_shards_rejected_on_every_rank():
    """A halo deeper than the thinnest shard raises at construction on EVERY rank
    (the same frame_height // world test everywhere), before any P2P call: uneven
    shards must not let some ranks enter the exchange while others raise."""
    from various_image_processings_amd.sharded import SlabGeometry
    for rank in range(2):
        with pytest.raises(ValueError):
            SlabGeometry(64, 29, 15, rank, 2)  # shards of 15 and 14 rows, halo 15
    SlabGeometry(64, 30, 15, 1, 2)  # 15 / 15: fine
    SlabGeometry(64, 5, 15, 0, 1)   # one rank: no halo exchange


def _split_worker(rank, world, port, width, height, ksize, kind, out_dir):
    """The interior band is filtered BEFORE the exchange (halo rows still garbage), the
    edge bands after it (sharded.split_bands, the order vip_shard_run and
    ShardedBilateral.filter use): equal to the full frame only if the interior reads
    no halo row."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import oracle as o
    from various_image_processings_amd.sharded import SlabGeometry, exchange_halo, split_bands

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frame = o.random_image(width, height)
    geo = SlabGeometry(width, height, ksize // 2, rank, world)
    b, e = geo.rows
    r = geo.radius
    slab = torch.full((geo.slab_rows, width, 3), 201, dtype=torch.uint8)  # garbage halos
    slab[r:r + geo.own] = torch.from_numpy(frame[b:e])
    lo, hi = geo.clamp_range()
    fn = o.adaptive_rows if kind == "adaptive" else o.bilateral_rows
    out = np.zeros((geo.own, width, 3), np.uint8)

    def band(row0, rows):
        if rows > 0:  # rows of the clamp-range view == the frame filter's rows
            view = np.ascontiguousarray(slab.numpy()[lo:hi])
            out[row0:row0 + rows] = fn(view, r + row0 - lo, rows, ksize)

    (i0, ni), edges = split_bands(geo)
    band(i0, ni)
    exchange_halo(slab, geo)
    for e0, ne in edges:
        band(e0, ne)
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,height,ksize,kind", [(2, 40, 9, "bilateral"), (3, 61, 7, "adaptive"),
                                                    (2, 20, 9, "bilateral")])  # (2, 20, 9): own 10 <= 2r, no interior
def test_interior_edge_split_matches_full_frame(tmp_path, world, height, ksize, kind):
    from oracle import oracle as o
    width = 23
    port = _free_port()
    mp.start_processes(_split_worker, args=(world, port, width, height, ksize, kind, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    got = np.concatenate([np.load(tmp_path / f"rank{i}.npy") for i in range(world)], axis=0)
    frame = o.random_image(width, height)
    want = (o.adaptive if kind == "adaptive" else o.bilateral)(frame, ksize)
    assert np.array_equal(got, want)


def test_split_bands_tile_the_own_rows():
    from various_image_processings_amd.sharded import SlabGeometry, split_bands
    for h in (16, 31, 100, 2160):
        for n in (1, 2, 3, 8):
            for r in (0, 1, 7, 15):
                if n > 1 and h // n < r:
                    continue
                for rank in range(n):
                    g = SlabGeometry(64, h, r, rank, n)
                    (i0, ni), edges = split_bands(g)
                    rows = sorted([(i0, ni)] + edges)
                    covered = [x for a, m in rows for x in range(a, a + m)]
                    assert covered == list(range(g.own)), (h, n, r, rank, rows)
                    if ni:
                        assert i0 - r >= 0 and i0 + ni + r <= g.own  # the interior's windows stay in own rows


class _InfoShard:
    """A stand-in for NativeShard.comm_info (what RCCL would report), for the gather logic."""

    def __init__(self, count, user_rank, bus):
        self.i = dict(count=count, user_rank=user_rank, device=0, pci_bus_id=bus)

    def comm_info(self):
        return dict(self.i)


def _rccl_worker(rank, world, port, mode, out_dir):
    import json
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import various_image_processings_amd.sharded as sh
    sh.rccl_version = lambda: 22606  # no RCCL call without a GPU
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bus = f"0000:{0x10 + rank:02x}:00.0" if mode != "same_device" else "0000:10:00.0"
    count = world if mode != "small_comm" else 1
    user = rank if mode != "small_comm" else 0
    ev = bench.rccl_evidence([_InfoShard(count, user, bus)] * 2, rank, world, world)
    with open(os.path.join(out_dir, f"rccl{rank}.json"), "w") as fh:
        json.dump(ev, fh)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["ok", "same_device", "small_comm"])
def test_rccl_evidence_gathered_over_gloo(tmp_path, mode):
    """bench.rccl_evidence at world size 2: every rank sees every rank's RCCL count, user rank
    and PCI bus id, and flags two ranks on one device or communicators of one rank each (what a
    line of an 8-GPU run that fell back or doubled up on a device would show)."""
    import json
    world = 2
    mp.spawn(_rccl_worker, args=(world, _free_port(), mode, str(tmp_path)), nprocs=world, join=True)
    evs = [json.load(open(tmp_path / f"rccl{r}.json")) for r in range(world)]
    assert evs[0] == evs[1]
    ev = evs[0]
    assert [r["rank"] for r in ev["ranks"]] == [0, 1]
    if mode == "ok":
        assert ev["problems"] == [] and ev["count"] == 2 and ev["distinct_devices"] == 2
    elif mode == "same_device":
        assert ev["distinct_devices"] == 1 and any("distinct devices" in p for p in ev["problems"])
    else:
        assert any("expected 2" in p for p in ev["problems"])
