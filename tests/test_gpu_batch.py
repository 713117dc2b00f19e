"""Multi-frame launches (include/vip.h vip_bilateral_run_rows_batch / vip_adaptive_run_rows_batch):
n frames of one geometry, up to 6 per launch, each frame bit-exact with its own run_rows call
and with the oracle. These launches carry a shard's B frames per RCCL group
(vip_shard_run_batch; tests/test_gpu_shard_native.py covers that path end to end)."""
import numpy as np
import pytest

from various_image_processings_amd._lib import VIP_ERR_ALIASING, VipError
from various_image_processings_amd.filters import _AdaptiveImpl, _BilateralImpl

pytestmark = pytest.mark.gpu


def _slabs(oracle, n, w, rows):
    return [oracle.random_u8(rows * w * 3).reshape(rows, w, 3) for _ in range(n)]


@pytest.mark.parametrize("kind,k", [("bilateral", 3), ("bilateral", 15), ("bilateral", 31), ("adaptive", 9),
                                    ("adaptive", 15)])
@pytest.mark.parametrize("n", [1, 2, 3, 6, 7])
def test_batch_equals_oracle_per_frame(dev, oracle, kind, k, n):
    """A 54-row slab per frame, 40 output rows centred 7 rows down, neighbours clamped to
    the slab: frame f's output is rows 7..46 of the oracle's filter of that slab. n = 7 is
    two launches (6 + 1)."""
    w, rows, out_rows, row0 = 200, 54, 40, 7
    imgs = _slabs(oracle, n, w, rows)
    impl = (_BilateralImpl if kind == "bilateral" else _AdaptiveImpl)(w, rows, k)
    srcs = [dev.put(x) for x in imgs]
    dsts = [dev.empty((out_rows, w, 3)) for _ in range(n)]
    impl.run_rows_batch(srcs, dsts, out_rows, row0, 0, rows)
    for f in range(n):
        want = (oracle.bilateral if kind == "bilateral" else oracle.adaptive)(imgs[f], k)[row0:row0 + out_rows]
        assert np.array_equal(dev.get(dsts[f]), want), f"frame {f} of {n}"


@pytest.mark.parametrize("kind", ["bilateral", "adaptive"])
@pytest.mark.parametrize("free_cus", [0, 16, 250, 10000])
def test_batch_small_slab_tiling(dev, oracle, kind, free_cus):
    """C2's slab at 8 GPUs (3840 x 270 own rows + two 7-row halos), 3 frames in one launch:
    the small-slab tiling is planned for all three frames' tiles, and the persistent
    workgroups leave free_cus CUs free (at least one workgroup runs: 10000 leaves one).
    Every frame equals its own run_rows launch; frame 0 equals the oracle."""
    w, r, own = 3840, 7, 270
    rows = own + 2 * r
    imgs = _slabs(oracle, 3, w, rows)
    impl = (_BilateralImpl if kind == "bilateral" else _AdaptiveImpl)(w, rows, 2 * r + 1)
    srcs = [dev.put(x) for x in imgs]
    dsts = [dev.empty((own, w, 3)) for _ in range(3)]
    impl.run_rows_batch(srcs, dsts, own, r, 0, rows, free_cus=free_cus)
    for f in range(3):
        one = dev.empty((own, w, 3))
        impl.run_rows(srcs[f], one, own, r, 0, rows)
        assert np.array_equal(dev.get(dsts[f]), dev.get(one)), f"frame {f}"
    want = (oracle.bilateral if kind == "bilateral" else oracle.adaptive)(imgs[0], 2 * r + 1)[r:r + own]
    assert np.array_equal(dev.get(dsts[0]), want)


def test_batch_unaligned_frame_and_runtime_radius(dev, oracle):
    """One frame at an odd byte address turns dword loads off for the whole launch; radius
    20 (the runtime-radius kernel) launches frame by frame. Both equal the oracle."""
    import torch
    w, rows = 131, 40
    imgs = _slabs(oracle, 3, w, rows)
    n = rows * w * 3
    big = torch.empty(4 * n + 16, dtype=torch.uint8, device="cuda")
    offs = [0, n + 1, 2 * n + 5]  # frames 1 and 2 unaligned
    for x, o in zip(imgs, offs):
        big[o:o + n].copy_(torch.from_numpy(x.reshape(-1)).cuda())
    srcs = [big.data_ptr() + o for o in offs]
    for k in (9, 41):
        impl = _BilateralImpl(w, rows, k)
        dsts = [dev.empty((rows, w, 3)) for _ in range(3)]
        impl.run_rows_batch(srcs, dsts, rows, 0, 0, rows)
        torch.cuda.synchronize()
        for f in range(3):
            assert np.array_equal(dev.get(dsts[f]), oracle.bilateral(imgs[f], k)), f"k {k} frame {f}"


def test_batch_rejects_aliasing_and_handles_empty(dev, oracle):
    w, rows = 64, 20
    impl = _BilateralImpl(w, rows, 5)
    a, b = dev.put(oracle.random_u8(rows * w * 3).reshape(rows, w, 3)), dev.empty((rows, w, 3))
    c = dev.empty((rows, w, 3))
    with pytest.raises(VipError) as e:
        impl.run_rows_batch([a, b], [c, a], rows, 0, 0, rows)  # frame 1 writes frame 0's input
    assert e.value.code == VIP_ERR_ALIASING
    impl.run_rows_batch([], [], rows, 0, 0, rows)  # nothing to do
    with pytest.raises(ValueError):
        impl.run_rows_batch([a], [], rows, 0, 0, rows)


@pytest.mark.parametrize("kind,k,w,own,inflight", [("bilateral", 15, 3840, 270, 1), ("bilateral", 15, 3840, 270, 2),
                                                   ("adaptive", 15, 3840, 270, 0), ("bilateral", 5, 1000, 97, 1),
                                                   ("adaptive", 9, 1000, 97, 0)])
def test_batch_last_round_pieces(dev, oracle, kind, k, w, own, inflight):
    """A multi-frame launch cuts its last round's tiles into pieces of a tile's waves, so
    that more workgroups share that round (plan_tail, vip_stencil.hpp; the plain bilateral
    only with one frame in flight, forced here both ways). Swept over workgroup counts
    (free_cus) to get last rounds of many sizes and piece counts: every frame of a 6-frame
    launch equals its one-frame launch (which never cuts a tile), and frame 0 the oracle."""
    import various_image_processings_amd as vip
    if inflight:
        vip.set_bilateral_frames_in_flight(inflight)
    try:
        _last_round_pieces(dev, oracle, kind, k, w, own)
    finally:
        vip.set_bilateral_frames_in_flight(0)


def _last_round_pieces(dev, oracle, kind, k, w, own):
    r = k // 2
    rows = own + 2 * r
    imgs = _slabs(oracle, 6, w, rows)
    impl = (_BilateralImpl if kind == "bilateral" else _AdaptiveImpl)(w, rows, k)
    srcs = [dev.put(x) for x in imgs]
    want = []
    for f in range(6):
        one = dev.empty((own, w, 3))
        impl.run_rows(srcs[f], one, own, r, 0, rows)
        want.append(dev.get(one))
    assert np.array_equal(want[0], (oracle.bilateral if kind == "bilateral" else oracle.adaptive)(imgs[0], k)[r:r + own])
    for free in (0, 3, 8, 29, 64, 130, 200, 251, 255):
        dsts = [dev.empty((own, w, 3)) for _ in range(6)]
        impl.run_rows_batch(srcs, dsts, own, r, 0, rows, free_cus=free)
        for f in range(6):
            assert np.array_equal(dev.get(dsts[f]), want[f]), f"free_cus {free} frame {f}"
