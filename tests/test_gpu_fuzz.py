"""Seeded random sweep of the HIP filters against the oracle, bit for bit.

The targeted parity tests (test_gpu_parity.py, test_gpu_ksize.py, test_gpu_fullsize.py)
pin the reference's own inputs, every ksize and every BASELINE size; this sweep crosses the
parameters they vary one at a time: frame shape (1 to a few hundred pixels each way, odd
widths, widths that are not a multiple of any tile), ksize, sigma_space, sigma_color (both
drawn over decades), the numerics profile, the input statistics (uniform, narrow
[100, 120) as sample/benchmark/main.cpp:213 uses, a smooth ramp), and -- through the C
ABI's pitch argument -- row padding. 48 cases, each small enough for the oracle to finish
in well under a second; a second sweep drives the multi-frame launches (run_rows_batch: row
bands of 2-6 frames, free CUs, frames in flight, and so the cut last round). VIP_FUZZ_CASES /
VIP_FUZZ_BATCH_CASES widen the sweeps for a one-off run (profiles/r05_fuzz_wide.log), and
VIP_FUZZ_SEED draws other cases.
"""
import os

import numpy as np
import pytest

import various_image_processings_amd as vip
from various_image_processings_amd import _lib

pytestmark = pytest.mark.gpu

N_CASES = int(os.environ.get("VIP_FUZZ_CASES", 48))
N_BATCH_CASES = int(os.environ.get("VIP_FUZZ_BATCH_CASES", 24))
SEED0 = int(os.environ.get("VIP_FUZZ_SEED", 0))  # another draw of cases for a one-off run


def _case(i):
    r = np.random.default_rng(SEED0 + 1000 + i)
    kind = ["bilateral", "joint", "adaptive", "texture"][i % 4]
    h, w = int(r.integers(1, 160)), int(r.integers(1, 300))
    if kind == "texture":
        k = int(r.integers(1, 10))
        nitr = int(r.integers(1, 4))
        ss = sc = None
    else:
        k = int(r.choice([1, 3, 5, 7, 9, 11, 13, 15, 17, 21, 25, 31]))
        nitr = None
        ss = float(10 ** r.uniform(-0.5, 2.5))
        sc = float(10 ** r.uniform(-0.3, 2.3))
    profile = int(r.integers(0, 2))
    data = ["uniform", "narrow", "ramp"][int(r.integers(0, 3))]
    # extra bytes per row (the C ABI's pitch; vip_texture_run takes dense frames)
    pad = 0 if kind == "texture" else int(r.choice([0, 0, 1, 13, 64]))
    return dict(kind=kind, h=h, w=w, k=k, nitr=nitr, ss=ss, sc=sc, profile=profile, data=data, pad=pad,
                seed=SEED0 + 1000 + i)


def _image(c, salt=0):
    r = np.random.default_rng(c["seed"] * 7 + salt)
    h, w = c["h"], c["w"]
    if c["data"] == "narrow":
        return r.integers(100, 120, (h, w, 3), dtype=np.uint8)
    if c["data"] == "ramp":
        y, x = np.mgrid[0:h, 0:w]
        base = (x * 3 + y * 5 + salt * 17) % 256
        return np.stack([base, (base + 85) % 256, (255 - base)], axis=-1).astype(np.uint8)
    return r.integers(0, 255, (h, w, 3), dtype=np.uint8)


def _pitched(dev, img, pad):
    """img in a device buffer whose rows are pad bytes longer than w * 3."""
    h, w, _ = img.shape
    buf = dev.empty((h, w * 3 + pad))
    buf.fill_(0xA5)
    buf[:, :w * 3] = dev.put(img.reshape(h, w * 3))
    return buf


def _out_pitched(dev, h, w, pad):
    buf = dev.empty((h, w * 3 + pad))
    buf.fill_(0x5A)
    return buf


def _unpitch(dev, buf, h, w):
    a = dev.get(buf)
    return np.ascontiguousarray(a[:, :w * 3]).reshape(h, w, 3), a[:, w * 3:]


@pytest.mark.parametrize("i", range(N_CASES))
def test_random_case_bit_exact(dev, oracle, i):
    c = _case(i)
    h, w, k, pad = c["h"], c["w"], c["k"], c["pad"]
    numerics = vip.VIP_NUMERICS_CPP if c["profile"] else vip.VIP_NUMERICS_CUDA
    img = _image(c)
    pitch = w * 3 + pad
    src, dst = _pitched(dev, img, pad), _out_pitched(dev, h, w, pad)
    s = dev.torch_.cuda.current_stream().cuda_stream
    lib = _lib.lib()
    if c["kind"] in ("bilateral", "joint"):
        impl = vip.filters._BilateralImpl(w, h, k, c["ss"], c["sc"], numerics)
        if c["kind"] == "joint":
            g_img = _image(c, salt=1)
            guide = _pitched(dev, g_img, pad)
            _lib.check("vip_joint_bilateral_run", lib.vip_joint_bilateral_run(
                impl._h, src.data_ptr(), pitch, guide.data_ptr(), pitch, dst.data_ptr(), pitch, s))
            want = oracle.joint_bilateral(img, g_img, k, c["ss"], c["sc"], profile=c["profile"])
        else:
            _lib.check("vip_bilateral_run", lib.vip_bilateral_run(impl._h, src.data_ptr(), pitch, dst.data_ptr(), pitch, s))
            want = oracle.bilateral(img, k, c["ss"], c["sc"], profile=c["profile"])
    elif c["kind"] == "adaptive":
        impl = vip.filters._AdaptiveImpl(w, h, k, c["ss"], c["sc"], numerics)
        _lib.check("vip_adaptive_run", lib.vip_adaptive_run(impl._h, src.data_ptr(), pitch, dst.data_ptr(), pitch, s))
        want = oracle.adaptive(img, k, c["ss"], c["sc"], profile=c["profile"])
    else:
        impl = vip.filters._TextureImpl(w, h, k, c["nitr"], numerics)
        _lib.check("vip_texture_run", lib.vip_texture_run(impl._h, src.data_ptr(), dst.data_ptr(), s))
        want = oracle.texture(img, k, c["nitr"], profile=c["profile"])
    got, tail = _unpitch(dev, dst, h, w)
    d = np.argwhere(got != want)
    assert not len(d), f"{c}: {len(d)} mismatches, first {d[:3].tolist()}"
    assert (tail == 0x5A).all(), f"{c}: the row padding of the output was written"


def _batch_case(i):
    r = np.random.default_rng(SEED0 + 5000 + i)
    kind = ["bilateral", "adaptive"][i % 2]
    k = int(r.choice([1, 3, 5, 7, 9, 11, 13, 15, 17]))  # the multi-frame kernels' radii (<= 8)
    h, w = int(r.integers(1, 200)), int(r.integers(1, 700))
    row0 = int(r.integers(0, h))
    out_rows = int(r.integers(1, h - row0 + 1))
    return dict(kind=kind, k=k, h=h, w=w, row0=row0, out_rows=out_rows, n=int(r.integers(2, 7)),
                free=int(r.choice([0, 0, 8, 16, 64, int(r.integers(0, 256))])), inflight=int(r.integers(0, 3)),
                ss=float(10 ** r.uniform(-0.5, 2.5)), sc=float(10 ** r.uniform(-0.3, 2.3)),
                profile=int(r.integers(0, 2)), seed=SEED0 + 5000 + i)


@pytest.mark.parametrize("i", range(N_BATCH_CASES))
def test_random_batch_case_bit_exact(dev, oracle, i):
    """n frames in one multi-frame launch (include/vip.h vip_*_run_rows_batch), output rows
    [row0, row0 + out_rows) of each, neighbours clamped to the frame: each equals the
    oracle's filter of that frame, those rows."""
    c = _batch_case(i)
    numerics = vip.VIP_NUMERICS_CPP if c["profile"] else vip.VIP_NUMERICS_CUDA
    r = np.random.default_rng(c["seed"])
    imgs = [r.integers(0, 255, (c["h"], c["w"], 3), dtype=np.uint8) for _ in range(c["n"])]
    cls = vip.filters._BilateralImpl if c["kind"] == "bilateral" else vip.filters._AdaptiveImpl
    impl = cls(c["w"], c["h"], c["k"], c["ss"], c["sc"], numerics)
    srcs = [dev.put(x) for x in imgs]
    dsts = [dev.empty((c["out_rows"], c["w"], 3)) for _ in imgs]
    vip.set_bilateral_frames_in_flight(c["inflight"])
    try:
        impl.run_rows_batch(srcs, dsts, c["out_rows"], c["row0"], 0, c["h"], free_cus=c["free"])
    finally:
        vip.set_bilateral_frames_in_flight(0)
    fn = oracle.bilateral if c["kind"] == "bilateral" else oracle.adaptive
    for f, x in enumerate(imgs):
        want = fn(x, c["k"], c["ss"], c["sc"], profile=c["profile"])[c["row0"]:c["row0"] + c["out_rows"]]
        got = dev.get(dsts[f])
        d = np.argwhere(got != want)
        assert not len(d), f"{c} frame {f}: {len(d)} mismatches, first {d[:3].tolist()}"
