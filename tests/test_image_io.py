"""Image files of the sample drivers (samples/vip_image_io.hpp through
`samples/vip_filter convert`, which never touches the GPU).

read_image must give what cv::imread(path, IMREAD_COLOR) gives the reference's samples
(sample/bilateral_filter/main.cpp:20 and the other sample/*/main.cpp): dense BGR, alpha
dropped, gray replicated, palette expanded, 16-bit reduced to the high byte, 1/2/4-bit
gray scaled to 0..255. The PNG inputs here come from an independent encoder written in
this file (every colour type and bit depth, all five row filters, Adam7), from PIL, and
-- in this container only -- the reference's own sample images, whose decode must equal
tests/golden/lenna_bgr.npz (the fixture every lenna test uses).
"""
import os
import struct
import subprocess
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "samples", "vip_filter")
REF_IMAGES = "/root/reference/sample_image"

ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def _chunk(kind, body):
    return struct.pack(">I", len(body)) + kind + body + struct.pack(">I", zlib.crc32(kind + body) & 0xFFFFFFFF)


def _pack_rows(samples, depth):
    """samples: (h, w, spp) ints -> list of packed row byte strings."""
    h, w, spp = samples.shape
    rows = []
    for y in range(h):
        flat = samples[y].reshape(-1).astype(np.int64)
        if depth == 16:
            rows.append(flat.astype(">u2").tobytes())
        elif depth == 8:
            rows.append(flat.astype(np.uint8).tobytes())
        else:
            per = 8 // depth
            n = (len(flat) + per - 1) // per
            out = np.zeros(n, np.int64)
            for i, v in enumerate(flat):
                out[i // per] |= int(v) << (8 - depth * (i % per + 1))
            rows.append(out.astype(np.uint8).tobytes())
    return rows


def _filter_rows(rows, bpp, first_filter):
    """Row filters cycling 0..4 from first_filter (the encoder side of PNG section 9)."""
    out = b""
    prev = bytes(len(rows[0])) if rows else b""
    for i, row in enumerate(rows):
        ft = (first_filter + i) % 5
        cur = np.frombuffer(row, np.uint8).astype(np.int64)
        up = np.frombuffer(prev, np.uint8).astype(np.int64)
        left = np.concatenate([np.zeros(bpp, np.int64), cur])[: len(cur)]
        ul = np.concatenate([np.zeros(bpp, np.int64), up])[: len(up)]
        if ft == 0:
            pred = np.zeros_like(cur)
        elif ft == 1:
            pred = left
        elif ft == 2:
            pred = up
        elif ft == 3:
            pred = (left + up) >> 1
        else:
            p = left + up - ul
            pa, pb, pc = np.abs(p - left), np.abs(p - up), np.abs(p - ul)
            pred = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, up, ul))
        out += bytes([ft]) + ((cur - pred) & 0xFF).astype(np.uint8).tobytes()
        prev = row
    return out


def encode_png(samples, ctype, depth, interlace=False, palette=None, first_filter=0):
    h, w, spp = samples.shape
    bpp = max(1, spp * depth // 8)
    raw = b""
    if interlace:
        for k, (x0, y0, dx, dy) in enumerate(ADAM7):
            sub = samples[y0::dy, x0::dx]
            if sub.shape[0] == 0 or sub.shape[1] == 0:
                continue
            raw += _filter_rows(_pack_rows(sub, depth), bpp, first_filter + k)
    else:
        raw = _filter_rows(_pack_rows(samples, depth), bpp, first_filter)
    png = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, int(interlace)))
    if palette is not None:
        png += _chunk(b"PLTE", palette.astype(np.uint8).tobytes())
        png += _chunk(b"tRNS", bytes(range(len(palette))))  # ignored: IMREAD_COLOR drops alpha
    png += _chunk(b"tEXt", b"Comment\x00ancillary chunk, skipped")
    z = zlib.compress(raw, 9)
    png += _chunk(b"IDAT", z[: len(z) // 2]) + _chunk(b"IDAT", z[len(z) // 2:])  # split IDAT
    return png + _chunk(b"IEND", b"")


def expected_bgr(samples, ctype, depth, palette=None):
    s = samples.astype(np.int64)
    if depth == 16:
        s = s >> 8
    elif depth < 8 and ctype == 0:
        s = s * 255 // ((1 << depth) - 1)
    if ctype == 3:
        return palette[s[..., 0]][..., ::-1].astype(np.uint8)
    if ctype in (0, 4):
        return np.repeat(s[..., :1], 3, axis=2).astype(np.uint8)
    return s[..., 2::-1].astype(np.uint8)


def read_ppm(path):
    b = open(path, "rb").read()
    parts = b.split(b"\n", 3)
    assert parts[0] in (b"P6", b"P5")
    w, h = map(int, parts[1].split())
    assert parts[2] == b"255"
    c = 3 if parts[0] == b"P6" else 1
    return np.frombuffer(parts[3], np.uint8).reshape(h, w, c)


def run(*args, ok=True):
    assert os.path.exists(EXE), "samples/vip_filter missing: run __graft_entry__.build() first"
    r = subprocess.run([EXE, *map(str, args)], capture_output=True, text=True, timeout=60)
    if ok:
        assert r.returncode == 0, r.stdout + r.stderr
    return r


def decode(tmp_path, png_bytes, name="in.png"):
    src = tmp_path / name
    src.write_bytes(png_bytes)
    run("convert", src, tmp_path / "out.ppm")
    return read_ppm(tmp_path / "out.ppm")[..., ::-1]  # PPM is RGB; back to BGR


CASES = [  # (ctype, depth, spp)
    (0, 1, 1), (0, 2, 1), (0, 4, 1), (0, 8, 1), (0, 16, 1),
    (2, 8, 3), (2, 16, 3),
    (3, 1, 1), (3, 2, 1), (3, 4, 1), (3, 8, 1),
    (4, 8, 2), (4, 16, 2),
    (6, 8, 4), (6, 16, 4),
]


@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("ctype,depth,spp", CASES)
def test_png_decode_every_format(tmp_path, ctype, depth, spp, interlace):
    rng = np.random.default_rng(ctype * 100 + depth + 7 * interlace)
    h, w = 13, 19  # ragged: partial bytes per row at low depths, empty Adam7 passes at 1 column
    palette = None
    hi = 1 << depth
    if ctype == 3:
        palette = rng.integers(0, 256, (hi, 3))
    samples = rng.integers(0, hi, (h, w, spp))
    for first in (0, 3):
        got = decode(tmp_path, encode_png(samples, ctype, depth, interlace, palette, first_filter=first))
        np.testing.assert_array_equal(got, expected_bgr(samples, ctype, depth, palette))


@pytest.mark.parametrize("shape", [(1, 1), (1, 9), (9, 1), (7, 8), (8, 8)])
def test_png_decode_tiny_interlaced(tmp_path, shape):
    rng = np.random.default_rng(shape[0] * 31 + shape[1])
    samples = rng.integers(0, 256, (*shape, 3))
    got = decode(tmp_path, encode_png(samples, 2, 8, interlace=True))
    np.testing.assert_array_equal(got, expected_bgr(samples, 2, 8))


def test_png_write_roundtrip_pil(tmp_path):
    PIL = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(5)
    bgr = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    bgr[10:20] = 128  # flat rows favour other row filters than noise does
    ppm = tmp_path / "in.ppm"
    ppm.write_bytes(b"P6\n# comment line\n53 37\n255\n" + bgr[..., ::-1].tobytes())
    run("convert", ppm, tmp_path / "out.png")
    np.testing.assert_array_equal(np.asarray(PIL.open(tmp_path / "out.png"))[..., ::-1], bgr)
    # and PIL-written PNGs (its own encoder's filters) decode to what PIL decodes
    for mode in ("RGB", "RGBA", "L", "P"):
        im = PIL.fromarray(bgr[..., ::-1]).convert(mode)
        im.save(tmp_path / f"pil_{mode}.png")
        got = decode(tmp_path, (tmp_path / f"pil_{mode}.png").read_bytes(), f"x_{mode}.png")
        np.testing.assert_array_equal(got, np.asarray(im.convert("RGB"))[..., ::-1])


def test_pnm_16bit_gray(tmp_path):
    rng = np.random.default_rng(9)
    g = rng.integers(0, 65536, (6, 11)).astype(">u2")
    p = tmp_path / "g.pgm"
    p.write_bytes(b"P5 11 6 65535\n" + g.tobytes())
    run("convert", p, tmp_path / "o.ppm")
    np.testing.assert_array_equal(read_ppm(tmp_path / "o.ppm")[..., 0], (g.astype(np.int64) >> 8).astype(np.uint8))


def test_corrupt_inputs_are_rejected(tmp_path):
    good = encode_png(np.zeros((4, 4, 3), np.int64), 2, 8)
    bad_crc = bytearray(good)
    bad_crc[40] ^= 0xFF  # inside IHDR/first chunk body or CRC
    cases = {"crc.png": bytes(bad_crc), "short.png": good[:-20], "text.png": b"hello", "empty.png": b""}
    for name, data in cases.items():
        (tmp_path / name).write_bytes(data)
        r = run("convert", tmp_path / name, tmp_path / "o.ppm", ok=False)
        assert r.returncode == 1 and "Failed to load" in r.stderr, (name, r.stderr)
    r = run("convert", tmp_path / "missing.png", tmp_path / "o.ppm", ok=False)
    assert r.returncode == 1
    r = run("nosuchfilter", tmp_path / "crc.png", tmp_path / "o.ppm", ok=False)
    assert r.returncode == 1


@pytest.mark.skipif(not os.path.isdir(REF_IMAGES), reason="reference sample images only exist in the build container")
def test_reference_lenna_decodes_to_fixture(tmp_path, lenna):
    got = decode(tmp_path, open(os.path.join(REF_IMAGES, "lenna.png"), "rb").read())
    np.testing.assert_array_equal(got, lenna)
