"""The native row-sharding path (include/vip_shard.h, libvip_shard.so) on the GPU.

Sharded output must equal one single-GPU launch over the whole frame, bit for bit:
* LOCAL transport: n slabs of one frame on the one device, halos by device copies,
  with the same split (interior rows while the halos move, then the edge bands) and
  the same stream ordering as the RCCL transport;
* RCCL transport with one rank (no neighbours; a one-device communicator), both as a
  one-process group and through the multi-process entry point with a unique id;
* a communicator whose peer never joins returns VIP_ERR_COMM_TIMEOUT, no hang;
* the texture filter (vip_shard_create_*_texture): one nitr-deep exchange per frame.
A multi-rank RCCL exchange needs several GPUs: it runs in the driver's 8-GPU bench.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import various_image_processings_amd as vip
from various_image_processings_amd import _shard_lib as S
from various_image_processings_amd.sharded import NativeShard, ShardGroup, native_unique_id, texture_halo_rows

pytestmark = pytest.mark.gpu


def _single(dev, img, k, adaptive, nitr=None):
    h, w, _ = img.shape
    d = dev.empty((h, w, 3))
    if nitr is not None:
        vip.CudaBilateralTextureFilter(w, h, k, nitr).execute(dev.put(img), d)
    elif adaptive:
        vip.CudaAdaptiveBilateralFilter(w, h, k).execute(dev.put(img), d)
    else:
        vip.CudaBilateralFilter(w, h, k).bilateral_filter(dev.put(img), d)
    return dev.get(d)


def _run_group(dev, img, k, n, adaptive, transport=S.VIP_SHARD_LOCAL, devices=None, split=True, nitr=None):
    torch = dev.torch_
    h, w, _ = img.shape
    g = ShardGroup(n, w, h, k, transport=transport, devices=devices, adaptive=adaptive, nitr=nitr)
    if nitr is None:
        g.set_split(split)
    slabs, outs, streams = [], [], []
    for geo in g.geos:
        b, e = geo.rows
        slab = dev.empty((geo.slab_rows, w, 3))
        slab.fill_(77)  # the halos are overwritten by the exchange (or unread at the frame edges)
        slab[geo.radius:geo.radius + geo.own] = dev.put(img[b:e])
        slabs.append(slab)
        outs.append(dev.empty((geo.own, w, 3)))
        streams.append(torch.cuda.Stream())
    torch.cuda.synchronize()
    g.filter(slabs, outs, streams)
    torch.cuda.synchronize()
    return np.concatenate([dev.get(o) for o in outs])


@pytest.mark.parametrize("n", [1, 2, 3, 8])
@pytest.mark.parametrize("adaptive", [False, True])
def test_local_group_equals_single_launch_4k(dev, oracle, n, adaptive):
    img = oracle.random_image(3840, 2160)
    want = _single(dev, img, 15, adaptive)
    for split in (True, False):
        got = _run_group(dev, img, 15, n, adaptive, split=split)
        assert np.array_equal(got, want), split


@pytest.mark.parametrize("shape,k,n", [((530, 700), 31, 8), ((77, 300), 9, 5), ((40, 131), 15, 5), ((64, 129), 65, 2)])
def test_local_group_ragged_vs_oracle(dev, oracle, shape, k, n):
    """Uneven shards (sizes differ by one), thin shards (own < 2r: no interior rows),
    the runtime-radius kernel (k = 65), against the oracle."""
    h, w = shape
    img = oracle.random_u8(h * w * 3).reshape(h, w, 3)
    got = _run_group(dev, img, k, n, False)
    assert np.array_equal(got, oracle.bilateral(img, k))


def test_local_group_c5_frame_8_way(dev, oracle):
    """C5's ksize 31 over a 16384-wide frame, 8 slabs: every pixel equals one launch."""
    img = oracle.random_image(16384, 2048)
    assert np.array_equal(_run_group(dev, img, 31, 8, False), _single(dev, img, 31, False))


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_local_group_texture_equals_single_run_4k(dev, oracle, n):
    """The texture filter row-sharded natively (vip_shard_create_group_texture): one
    45-row halo exchange per frame (k = 5, nitr = 5), a shrinking ghost zone over the
    iterations; every pixel equals one vip_texture_run of the whole 4K frame."""
    img = oracle.random_image(3840, 2160)
    assert np.array_equal(_run_group(dev, img, 5, n, False, nitr=5), _single(dev, img, 5, False, nitr=5))


@pytest.mark.parametrize("shape,k,nitr,n", [((301, 173), 5, 3, 3), ((200, 150), 4, 2, 2), ((90, 120), 3, 1, 4),
                                            ((64, 80), 5, 0, 2), ((130, 97), 9, 2, 2)])
def test_local_group_texture_vs_oracle(dev, oracle, shape, k, nitr, n):
    """Ragged frames, an even k, one iteration, nitr = 0 (the source), against the oracle."""
    h, w = shape
    img = oracle.random_u8(h * w * 3).reshape(h, w, 3)
    assert np.array_equal(_run_group(dev, img, k, n, False, nitr=nitr), oracle.texture(img, k, nitr))


def test_texture_shard_has_no_split(dev):
    g = ShardGroup(2, 256, 200, 5, nitr=2)
    assert g.geos[0].radius == 2 * 9
    with pytest.raises(vip.VipError) as e:
        g.set_split(True)
    assert e.value.code == 10001
    with pytest.raises(vip.VipError):
        ShardGroup(8, 256, 300, 5, nitr=5)  # 37-row shards < 45-row halo


def test_rccl_texture_single_rank(dev, oracle):
    """vip_shard_create_texture with a unique id, nranks = 1, and a one-device group."""
    import torch
    img = oracle.random_image(700, 400)
    want = _single(dev, img, 5, False, nitr=3)
    s = NativeShard(700, 400, 5, 0, 1, native_unique_id(), nitr=3)
    geo = s.geo
    slab = dev.empty((geo.slab_rows, 700, 3))
    slab[geo.radius:geo.radius + geo.own] = dev.put(img)
    out = dev.empty((400, 700, 3))
    s.filter(slab, out)
    torch.cuda.synchronize()
    assert np.array_equal(dev.get(out), want)
    got = _run_group(dev, img, 5, 1, False, transport=S.VIP_SHARD_RCCL, devices=[torch.cuda.current_device()], nitr=3)
    assert np.array_equal(got, want)


def test_thin_shards_rejected_before_any_device_work(dev):
    with pytest.raises(vip.VipError) as e:
        ShardGroup(8, 64, 100, 31)  # 12-row shards < 15-row halo
    assert e.value.code == 10001


@pytest.mark.parametrize("adaptive", [False, True])
def test_rccl_one_device_group(dev, oracle, adaptive):
    import torch
    img = oracle.random_image(1000, 600)
    got = _run_group(dev, img, 15, 1, adaptive, transport=S.VIP_SHARD_RCCL, devices=[torch.cuda.current_device()])
    assert np.array_equal(got, _single(dev, img, 15, adaptive))


def test_rccl_single_rank_native_shard_timed(dev, oracle):
    """vip_shard_create with a unique id and nranks = 1 (the multi-process entry point),
    vip_shard_run and vip_shard_run_timed: equal to one launch; events in order."""
    torch = dev.torch_
    img = oracle.random_image(900, 500)
    s = NativeShard(900, 500, 15, 0, 1, native_unique_id())
    geo = s.geo
    slab = dev.empty((geo.slab_rows, 900, 3))
    slab[geo.radius:geo.radius + geo.own] = dev.put(img)
    out = dev.empty((500, 900, 3))
    s.filter(slab, out)
    want = _single(dev, img, 15, False)
    assert np.array_equal(dev.get(out), want)
    for split in (True, False):
        s.set_split(split)
        out.zero_()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        s.filter_timed(slab, out, ev)
        torch.cuda.synchronize()
        assert np.array_equal(dev.get(out), want)
        assert ev[0].elapsed_time(ev[3]) > 0


def test_rccl_single_rank_batch(dev, oracle):
    """vip_shard_run_batch on a one-rank communicator: three frames (different images) in
    one call, each equal to its own single launch, in both split modes."""
    img = [oracle.random_image(900, 500) if f == 0 else np.ascontiguousarray(oracle.random_image(900, 500)[::-1])
           for f in range(2)]
    img.append(np.ascontiguousarray(img[0][:, ::-1]))
    s = NativeShard(900, 500, 15, 0, 1, native_unique_id())
    geo = s.geo
    slabs, outs = [], []
    for im in img:
        sl = dev.empty((geo.slab_rows, 900, 3))
        sl[geo.radius:geo.radius + geo.own] = dev.put(im)
        slabs.append(sl)
        outs.append(dev.empty((500, 900, 3)))
    run = s.batch_launcher()
    for split in (True, False):
        s.set_split(split)
        for o in outs:
            o.zero_()
        run([t.data_ptr() for t in slabs], [t.data_ptr() for t in outs], dev.torch_.cuda.current_stream().cuda_stream)
        dev.torch_.cuda.synchronize()
        for im, o in zip(img, outs):
            assert np.array_equal(dev.get(o), _single(dev, im, 15, False))


def test_rccl_missing_peer_times_out():
    """A 2-rank communicator whose second rank never joins: vip_shard_create returns
    VIP_ERR_COMM_TIMEOUT after its timeout instead of blocking (run in a child process
    with its own limit, so a hang could not stall the suite)."""
    code = r'''
import ctypes, sys, time
sys.path.insert(0, sys.argv[1])
from various_image_processings_amd import _shard_lib as S
from various_image_processings_amd.sharded import native_unique_id
h = ctypes.c_void_p()
t0 = time.time()
rc = S.lib().vip_shard_create(ctypes.byref(h), 0, 64, 64, 3, 10.0, 30.0, 0, 2, 0,
                              ctypes.create_string_buffer(native_unique_id(), 128), 3000)
print(rc, round(time.time() - t0, 1), S.lib().vip_shard_last_error().decode(), flush=True)
import os
os._exit(0)  # RCCL's bootstrap thread still waits for the missing rank: leave without joining it
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, NCCL_DEBUG="WARN")
    r = subprocess.run([sys.executable, "-c", code, root], capture_output=True, text=True, timeout=90, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    rc, secs = r.stdout.strip().splitlines()[-1].split()[:2]  # RCCL prints its banner first
    assert int(rc) == S.VIP_ERR_COMM_TIMEOUT, r.stdout
    assert 2.5 <= float(secs) < 60, r.stdout


@pytest.mark.parametrize("argv", [["4096", "2048", "31", "2", "--local", "8"], ["3840", "2160", "15", "3"],
                                  ["2000", "999", "63", "1", "--local", "3", "--adaptive"],
                                  ["3840", "2160", "5", "2", "--local", "4", "--texture", "5"]])
def test_shard_frame_sample(dev, argv):
    """samples/vip_shard_frame (a C++ caller of vip_shard.h): the sharded frame gathered
    from its shards equals one whole-frame launch (exit status 0, 'equals')."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "samples", "vip_shard_frame")
    assert os.path.exists(exe), "build first"
    r = subprocess.run([exe] + argv, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "equals the one-launch output" in r.stdout, r.stdout + r.stderr[-2000:]


# --- loopback transport: the RCCL neighbour path on one GPU --------------------------
# vip_shard_create_loopback: the shard's row neighbours are itself over a one-rank
# communicator, so enqueue_p2p's ncclSend/ncclRecv pairs, the group end, the ev_in / ev_x
# ordering, the batch group and graph capture all run for real. The halo above receives
# the shard's own top r rows and the halo below its own bottom r rows, so the expected
# output is the filter of that slab taken as a frame, on the own rows.
def _loopback_frame(img, r, rank, n):
    parts = [img[:r]] if rank > 0 else []
    parts.append(img)
    if rank < n - 1:
        parts.append(img[-r:])
    return np.ascontiguousarray(np.concatenate(parts)), (r if rank > 0 else 0)


def _loopback_slab(dev, s, img):
    geo = s.geo
    slab = dev.empty((geo.slab_rows, img.shape[1], 3))
    slab.fill_(201)  # the exchange overwrites the halos it owns
    slab[geo.radius:geo.radius + geo.own] = dev.put(img)
    return slab


def _loopback_want(dev, img, k, rank, n, adaptive=False, nitr=None):
    r = k // 2 if nitr is None else nitr * texture_halo_rows(k)
    frame, top = _loopback_frame(img, r, rank, n)
    return _single(dev, frame, k, adaptive, nitr)[top:top + img.shape[0]]


@pytest.mark.parametrize("rank", [0, 1, 2])
@pytest.mark.parametrize("adaptive", [False, True])
def test_loopback_rccl_exchange(dev, oracle, rank, adaptive):
    torch = dev.torch_
    w, own = 1000, 300
    img = oracle.random_image(w, own)
    s = NativeShard(w, 3 * own, 15, rank, 3, None, adaptive=adaptive, loopback=True)
    assert s.geo.own == own
    want = _loopback_want(dev, img, 15, rank, 3, adaptive)
    for split in (True, False, True):
        s.set_split(split)
        slab = _loopback_slab(dev, s, img)
        out = dev.empty((own, w, 3))
        s.filter(slab, out)
        torch.cuda.synchronize()
        assert np.array_equal(dev.get(out), want), split


def test_loopback_against_the_oracle(dev, oracle):
    w, own = 131, 40
    img = oracle.random_u8(w * own * 3).reshape(own, w, 3)
    s = NativeShard(w, 3 * own, 9, 1, 3, None, loopback=True)
    s.set_split(True)
    slab = _loopback_slab(dev, s, img)
    out = dev.empty((own, w, 3))
    s.filter(slab, out)
    dev.torch_.cuda.synchronize()
    frame, top = _loopback_frame(img, 4, 1, 3)
    assert np.array_equal(dev.get(out), oracle.bilateral(frame, 9)[top:top + own])


def test_loopback_timed_events_in_order(dev, oracle):
    """split 0: events[2] is recorded once the filter stream has the halos (after the wait),
    so it is not earlier than the exchange's end (events[1]); split 1: after the interior."""
    torch = dev.torch_
    w, own = 3840, 270
    img = oracle.random_image(w, own)
    s = NativeShard(w, 8 * own, 15, 3, 8, None, loopback=True)
    want = _loopback_want(dev, img, 15, 3, 8)
    slab = _loopback_slab(dev, s, img)
    out = dev.empty((own, w, 3))
    s.filter(slab, out)  # the first exchange connects the peer
    for split in (False, True):
        s.set_split(split)
        for _ in range(3):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            out.zero_()
            s.filter_timed(slab, out, ev)
            torch.cuda.synchronize()
            assert np.array_equal(dev.get(out), want)
            t1, t2, t3 = (ev[0].elapsed_time(ev[j]) for j in (1, 2, 3))
            assert 0 <= t2 <= t3 and t1 <= t3
            if not split:
                assert t1 <= t2 + 1e-3


@pytest.mark.parametrize("split,shared", [(False, None), (True, None), (False, 0), (False, 16)])
@pytest.mark.parametrize("adaptive", [False, True])
def test_loopback_batch(dev, oracle, split, shared, adaptive):
    """vip_shard_run_batch with neighbours: the halos of three frames in one RCCL group;
    shared (not None): the three frames filtered in one launch leaving that many CUs free
    (vip_shard_set_frames_launch)."""
    torch = dev.torch_
    w, own = 900, 200
    imgs = [oracle.random_image(w, own), np.ascontiguousarray(oracle.random_image(w, own)[::-1])]
    imgs.append(np.ascontiguousarray(imgs[0][:, ::-1]))
    s = NativeShard(w, 4 * own, 15, 2, 4, None, adaptive=adaptive, loopback=True)
    s.set_split(split)
    s.set_frames_launch(shared is not None, shared or 0)
    slabs = [_loopback_slab(dev, s, im) for im in imgs]
    outs = [dev.empty((own, w, 3)) for _ in imgs]
    s.batch_launcher()([t.data_ptr() for t in slabs], [t.data_ptr() for t in outs],
                       torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for im, o in zip(imgs, outs):
        assert np.array_equal(dev.get(o), _loopback_want(dev, im, 15, 2, 4, adaptive))


@pytest.mark.parametrize("argv", [[], ["--split"], ["1200", "300", "5", "3", "--texture", "5"],
                                  ["2000", "700", "31", "8"], ["--fail-capture"]])
def test_loopback_graph_replay_cpp(argv):
    """Graph mode (vip_shard_set_graph) from C++ (tests/cpp/shard_graph_test, outside torch):
    loopback shards, one per stream, two frames in flight; every frame replayed from its
    captured graph equals its direct run (exit 0). Also prints host enqueue time per frame,
    direct against graph. Run in a child process with its own limit."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tests", "cpp", "shard_graph_test")
    assert os.path.exists(exe), "build first"
    r = subprocess.run([exe] + argv, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "graph frames equal the direct frames" in r.stdout, r.stdout + r.stderr[-3000:]
    if "--fail-capture" in argv:
        # every capture failed: each frame still ran directly (its exchange included), graph
        # mode switched itself off, and the library said so
        assert "fell back to direct frames" in r.stdout and "graph capture failed" in r.stderr
    else:
        assert "graphs dropped after their streams were destroyed" in r.stdout


def test_comm_info_one_rank_and_loopback(dev):
    """vip_shard_comm_info: RCCL's own count / user rank / device of a shard's communicator.
    A one-rank shard and a loopback shard (one-rank communicator, itself as neighbours) both
    report 1 / 0 / the current device, and the device's PCI bus id."""
    torch = dev.torch_
    cur = torch.cuda.current_device()
    for s in (NativeShard(900, 500, 15, 0, 1, native_unique_id()), NativeShard(900, 4 * 200, 15, 2, 4, None,
                                                                             loopback=True)):
        info = s.comm_info()
        assert (info["count"], info["user_rank"], info["device"]) == (1, 0, cur), info
        bus = info["pci_bus_id"]
        assert len(bus.split(":")) == 3 and "." in bus, bus
        s.close()


def test_graph_mode_refused_below_the_verified_rccl(dev):
    """vip_shard_set_graph refuses graph mode (VIP_ERR_UNSUPPORTED) when the RCCL bound in
    this process is older than 2.27.7 -- in a torch process that is torch's bundled copy,
    whose capture of a send/recv group crashes -- and accepts it otherwise."""
    from various_image_processings_amd.sharded import rccl_version
    v = rccl_version()
    assert v > 20000, v
    s = NativeShard(900, 4 * 200, 15, 2, 4, None, loopback=True)
    if v < S.GRAPH_MIN_RCCL_VERSION:
        with pytest.raises(S.ShardError) as e:
            s.set_graph(True)
        assert e.value.code == S.VIP_ERR_UNSUPPORTED and "2.27.7" in str(e.value)
        assert s.graph_count() == 0
    else:
        s.set_graph(True)
    s.set_graph(False)  # turning it off is always allowed
    s.close()
