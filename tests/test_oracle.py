"""CPU tests of the oracle (test infrastructure): pinned inputs, regression
goldens, and an independent numpy restatement on small cases."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT


@pytest.mark.parametrize("name,kind,n,mx", [
    ("random_array_u8_7500_255.bin", "u8", 7500, 255),
    ("random_array_u8_2500_255.bin", "u8", 2500, 255),
    ("random_array_f32_2500_255.bin", "f32", 2500, 255.0),
    ("random_array_f32_7500_255.bin", "f32", 7500, 255.0),
    ("random_array_f32_2500_1.bin", "f32", 2500, 1.0),
])
def test_input_generator_pinned_to_reference(oracle, name, kind, n, mx):
    """oracle mt19937 == the reference's test/random_array.hpp (compiled in place)."""
    ref = open(os.path.join(GOLDEN, name), "rb").read()
    if kind == "u8":
        assert np.array_equal(np.frombuffer(ref, np.uint8), oracle.random_u8(n, mx))
    else:
        assert np.array_equal(np.frombuffer(ref, np.float32), oracle.random_f32(n, mx))


def test_oracle_regression_goldens(oracle, goldens, lenna):
    import hashlib
    img = oracle.random_image(50, 50)
    for prof, tag in ((oracle.CUDA, "cuda"), (oracle.CPP, "cpp")):
        for k in (3, 9, 11, 15, 31):
            assert np.array_equal(goldens[f"bilateral_{tag}_k{k}"], oracle.bilateral(img, k, 10.0, 30.0, prof))
            assert np.array_equal(goldens[f"adaptive_{tag}_k{k}"], oracle.adaptive(img, k, 10.0, 30.0, prof))
        sha = hashlib.sha256(oracle.bilateral(lenna, 11, 10.0, 30.0, prof, threads=4).tobytes()).digest()
        assert np.array_equal(goldens[f"lenna_bilateral_{tag}_k11_sha256"], np.frombuffer(sha, np.uint8))
        assert np.array_equal(goldens[f"texture_{tag}_k5_n5"], oracle.texture(oracle.random_image(64, 48), 5, 5, prof))


def test_threaded_oracle_equals_serial(oracle):
    img = oracle.random_image(97, 61)
    assert np.array_equal(oracle.bilateral(img, 11, threads=1), oracle.bilateral(img, 11, threads=5))
    assert np.array_equal(oracle.adaptive(img, 9, threads=1), oracle.adaptive(img, 9, threads=3))


def test_constant_image_is_fixed_point(oracle):
    c = np.full((13, 21, 3), (17, 200, 99), np.uint8)
    for prof in (oracle.CUDA, oracle.CPP):
        assert np.array_equal(oracle.bilateral(c, 9, profile=prof), c)
        assert np.array_equal(oracle.adaptive(c, 9, profile=prof), c)
        assert np.array_equal(oracle.texture(c, 5, 2, profile=prof), c)


def test_profiles_agree_within_one(oracle, lenna):
    """The reference's own GPU path (float LUT + fma) and CPU path (double LUT,
    mul+add) agree within the +-1 its tests allow (test/bilateral_filter.cu:58-60)."""
    crop = lenna[200:280, 200:300]
    for fn in (oracle.bilateral, oracle.adaptive):
        a = fn(crop, 11, profile=oracle.CUDA).astype(int)
        b = fn(crop, 11, profile=oracle.CPP).astype(int)
        assert np.abs(a - b).max() <= 1


# ---------------------------------------------------------------------------
# Independent numpy restatement (float32 arithmetic in the reference's order)
# cross-checks the C transcription on small images.
# ---------------------------------------------------------------------------
def _np_luts(ksize, ss, sc, n, profile):
    r = ksize // 2
    two_ss = np.float32(2) * np.float32(ss) * np.float32(ss)
    two_sc = np.float32(2) * np.float32(sc) * np.float32(sc)
    ky, kx = np.mgrid[-r:r + 1, -r:r + 1]
    r2 = kx * kx + ky * ky
    i = np.arange(n)
    if profile == 1:
        space = np.exp(r2.astype(np.float64) * (-1.0 / np.float64(two_ss))).astype(np.float32)
        color = np.exp((i * i).astype(np.float64) * (-1.0 / np.float64(two_sc))).astype(np.float32)
    else:
        space = np.exp(r2.astype(np.float32) * (np.float32(-1) / two_ss)).astype(np.float32)
        color = np.exp((i * i).astype(np.float32) * (np.float32(-1) / two_sc)).astype(np.float32)
    space[r2 > r * r] = 0
    return space, color


def _np_bilateral_cpp(src, ksize, ss=10.0, sc=30.0, guide=None):
    """include/cpp/bilateral_filter.hpp:76-104 in numpy float32, profile CPP."""
    g = src if guide is None else guide
    h, w, _ = src.shape
    r = ksize // 2
    space, color = _np_luts(ksize, ss, sc, 768, 1)
    s = np.zeros((h, w, 3), np.float32)
    sk = np.zeros((h, w), np.float32)
    ys, xs = np.arange(h), np.arange(w)
    for ky in range(-r, r + 1):
        yc = np.clip(ys + ky, 0, h - 1)
        for kx in range(-r, r + 1):
            xc = np.clip(xs + kx, 0, w - 1)
            nb = src[yc][:, xc].astype(np.float32)
            gq = g[yc][:, xc].astype(np.int32)
            d = np.abs(g.astype(np.int32) - gq).sum(axis=2)
            wgt = (space[ky + r, kx + r] * color[d]).astype(np.float32)
            s = (s + nb * wgt[..., None]).astype(np.float32)
            sk = (sk + wgt).astype(np.float32)
    return (s / sk[..., None] + np.float32(0.5)).astype(np.float32).astype(np.int32).astype(np.uint8)


def test_numpy_restatement_bilateral_cpp(oracle):
    img = oracle.random_image(23, 17)
    guide = oracle.random_image(17, 23).reshape(17, 23, 3)[:, ::-1].copy()
    for k in (3, 9):
        assert np.array_equal(_np_bilateral_cpp(img, k), oracle.bilateral(img, k, profile=oracle.CPP))
        assert np.array_equal(_np_bilateral_cpp(img, k, guide=guide),
                              oracle.joint_bilateral(img, guide, k, profile=oracle.CPP))


def test_numpy_restatement_gradient(oracle):
    for ch in (1, 3):
        u8 = oracle.random_u8(40 * 30 * ch).reshape(30, 40, ch)
        f = oracle.random_f32(40 * 30 * ch).reshape(30, 40, ch)
        for a in (u8, f):
            x = a.astype(np.float32)
            xp = np.concatenate([x[:, 1:], x[:, -1:]], 1)
            xm = np.concatenate([x[:, :1], x[:, :-1]], 1)
            yp = np.concatenate([x[1:], x[-1:]], 0)
            ym = np.concatenate([x[:1], x[:-1]], 0)
            h, v = (xp - xm).astype(np.float32), (yp - ym).astype(np.float32)
            # CPP profile: sum_c (h*h + v*v)
            s = np.zeros(x.shape[:2], np.float32)
            for c in range(ch):
                s = (s + ((h[..., c] * h[..., c]).astype(np.float32) + (v[..., c] * v[..., c]).astype(np.float32))
                     ).astype(np.float32)
            assert np.array_equal(np.sqrt(s), oracle.gradient(a, profile=oracle.CPP))


@pytest.mark.parametrize("k", [5, 4, 6])
def test_numpy_restatement_blur_rtv_guide(oracle, k):
    """Odd and EVEN k. Even k follows include/cpp/bilateral_texture_filter.hpp:41-59 and
    :98-101: the window is +-(k / 2), i.e. (k + 1) x (k + 1) taps, the box sum is divided
    by k * k and sigma_alpha is 1 / (5k). (The reference's CUDA stages use the same
    window but size their tile for k - 1 apron columns,
    src/bilateral_texture_filter_impl.cu:28,80-85: undefined there.)"""
    img = oracle.random_image(31, 19)
    mag = oracle.random_f32(31 * 19).reshape(19, 31)
    r = k // 2
    b, rtv = oracle.blur_rtv(img, mag, k, oracle.CUDA)
    h, w = mag.shape
    ys, xs = np.arange(h), np.arange(w)
    s = np.zeros((h, w, 3), np.float32)
    imax = np.zeros((h, w), np.float32)
    imin = np.full((h, w), 256, np.float32)
    mmax = np.zeros((h, w), np.float32)
    msum = np.zeros((h, w), np.float32)
    for ky in range(-r, r + 1):
        yc = np.clip(ys + ky, 0, h - 1)
        for kx in range(-r, r + 1):
            xc = np.clip(xs + kx, 0, w - 1)
            p = img[yc][:, xc]
            s = (s + p.astype(np.float32)).astype(np.float32)
            inten = (p.astype(np.int32).sum(2).astype(np.float32) / np.float32(3)).astype(np.float32)
            imax, imin = np.maximum(imax, inten), np.minimum(imin, inten)
            m = mag[yc][:, xc]
            mmax = np.maximum(mmax, m)
            msum = (msum + m).astype(np.float32)
    assert np.array_equal(b, (s / np.float32(k * k)).astype(np.float32))
    num = ((imax - imin) * mmax).astype(np.float32)
    assert np.array_equal(rtv, (num.astype(np.float64) / (msum.astype(np.float64) + 1e-9)).astype(np.float32))
    # guide: first strict argmin, alpha blend with fma (profile CUDA)
    g = oracle.guide(b, rtv, k, oracle.CUDA)
    sa = np.float32(1) / np.float32(5 * k)
    for y in range(h):
        for x in range(w):
            best, by, bx = np.float32(1e10), 0, 0
            for ky in range(-r, r + 1):
                for kx in range(-r, r + 1):
                    yy, xx = min(max(y + ky, 0), h - 1), min(max(x + kx, 0), w - 1)
                    if best > rtv[yy, xx]:
                        best, by, bx = rtv[yy, xx], yy, xx
            e = np.float32(np.exp(np.float64(np.float32(sa * np.float32(rtv[y, x] - best)))))
            alpha = np.float32(np.float32(2) / np.float32(1 + e)) - np.float32(1)
            beta = np.float32(1) - alpha
            for c in range(3):
                prod = np.float64(beta * b[y, x, c]).astype(np.float32)
                v = np.float32(np.float64(alpha) * np.float64(b[by, bx, c]) + np.float64(prod))  # exact fma
                v = np.float32(v + np.float32(0.5))
                assert g[y, x, c] == min(max(int(v), 0), 255), (y, x, c)


def _fma32(a, b, c):
    """float32 fma, exact through long double: every product/sum below spans < 64 bits."""
    ld = np.longdouble
    return (ld(a) * ld(b) + ld(c)).astype(np.float32)


@pytest.mark.skipif(np.finfo(np.longdouble).nmant < 63, reason="needs x87 80-bit long double")
def test_constant_division_is_exact():
    """The fused texture guide stage and the adaptive kernel (vip_stencil.hpp
    div_exact) divide integer box sums by ksize^2, and intensity byte sums by 3, with
    an fma-corrected reciprocal: q0 = s*rd, q = fma(fma(-q0, d, s), rd, q0). It must
    equal the correctly rounded float quotient the reference computes
    (src/bilateral_texture_filter_impl.cu:97-100, :84;
    src/adaptive_bilateral_filter_impl.cu:88-92) for EVERY reachable numerator --
    checked exhaustively here (texture ksize 2..24 and beyond, windows 2*(k//2)+1 wide for
    even k too; adaptive ksize up to 31 -- above, the runtime-radius kernel divides in IEEE)."""
    cases = [((2 * (k // 2) + 1) ** 2 * 255, k * k) for k in range(2, 32)] + [(765, 3)]
    for smax, d in cases:
        s = np.arange(smax + 1, dtype=np.float32)
        d32 = np.float32(d)
        rd = np.float32(1) / d32
        q0 = (s * rd).astype(np.float32)
        q = _fma32(_fma32(-q0, d32, s), rd, q0)
        assert np.array_equal(q, (s / d32).astype(np.float32)), d


def test_numerics_sensitivity_within_reference_tolerance():
    """The unpinned CUDA-profile choices (sumk add, guide-blend contraction, exp
    rounding -- oracle.VARIANTS) and the include/cpp numerics move the outputs by at
    most the reference tests' +-1 (test/bilateral_filter.cu:58-60) for the
    bilateral, joint and adaptive filters; the texture filter ("<= 1 on
    >= 99.9 %") stays within 1 on >= 99.9 % of channels. scripts/numerics_sensitivity.py
    writes the full table (profiles/r02_numerics_sensitivity.json)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ns", os.path.join(ROOT, "scripts", "numerics_sensitivity.py"))
    ns = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ns)
    from oracle import oracle as o
    for name, fn in ns.cases().items():
        base = fn(o.CUDA)
        alts = [("cpp", fn(o.CPP))]
        for vname, flags in o.VARIANTS.items():
            if vname.startswith(("blend", "exp")) and not name.startswith("texture"):
                continue
            with o.variant(flags):
                alts.append((vname, fn(o.CUDA)))
        for vname, alt in alts:
            s = ns.stats(alt, base)
            if name.startswith("texture"):
                assert s["within1_pct"] >= 99.9, (name, vname, s)
            else:
                assert s["max_abs"] <= 1, (name, vname, s)


def test_texture_rows_band_equals_full_frame(oracle):
    """oracle.texture_rows (a crop with an nitr * halo ghost margin) == those rows of
    the full-frame filter: the full-size GPU texture test relies on it."""
    img = oracle.random_image(61, 140)
    full = oracle.texture(img, 5, 3)
    for r0, n in ((0, 7), (50, 11), (131, 9)):
        assert np.array_equal(oracle.texture_rows(img, r0, n, 5, 3), full[r0:r0 + n])


def test_table_exp_equals_glibc_exp(tmp_path):
    """The texture guide's alpha uses a 64-entry-table double exp on the GPU
    (vip_stencil.hpp exp_tab_f32); microbench/exp_check restates it bit for bit (same table,
    constants and fma sequence) and compares it with glibc's (float)exp((double)x) -- the
    oracle's -- for EVERY float x in [0, 32), the whole range the argument can take.
    (div_check compares the device version with ocml's on the GPU.)"""
    import subprocess
    exe = tmp_path / "exp_check"
    src = os.path.join(ROOT, "microbench", "exp_check.c")
    inc = os.path.join(ROOT, "various_image_processings_amd", "csrc")
    subprocess.run(["cc", "-O2", "-ffp-contract=off", "-I", inc, "-o", str(exe), src, "-lm", "-lpthread"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and " 0 mismatches" in r.stdout, r.stdout + r.stderr
