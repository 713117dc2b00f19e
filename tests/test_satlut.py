"""The saturating colour-LUT address (SatLut, various_image_processings_amd/csrc/vip_stencil.hpp)
as integer arithmetic on the CPU.

The joint kernel (texture JBF, R <= 6) and the adaptive kernel address their LUT with one
v_mad_legacy_u16 carrying the clamp bit: reg = min(d*S + B0 + 4c, 65535), high half zero
(checked on gfx950 by microbench/sat_addr.hip, profiles/r03_sat_addr.txt), then ds_read at
reg + T - B0 + 128k (immediate). For every radius, every colour distance the kernels can form,
every lane copy c and every r^2 table k, this checks that the address lands on the word the
kernel means -- entry (d, k, c) while d <= DZ, the exact-zero entry (DZ, k, 31) beyond -- that
the colour LUT really is zero wherever saturation reads (both numerics profiles), that the
unsaturated lanes of a half-wave hit 32 distinct banks, and that tables, planes and the
immediate fit their ranges. The constants restate the constexpr formulas of SatLut and the
adaptive kernel (vip_adaptive.hip); the GPU tests check the outputs bit for bit.
"""
import numpy as np
import pytest

from oracle import oracle as o

LDS_BUDGET = 160 * 1024
SIGMA_TEXTURE = 1.73205080757  # the texture filter's JBF sigma_color (vip_capi.hip)


def round_up(v, m):
    return (v + m - 1) // m * m


def disc_r2_values(R):
    return sorted({x * x + y * y for x in range(R + 1) for y in range(R + 1) if x * x + y * y <= R * R})


def sat_layout(ntab, dzmax, plane_bytes):
    S = ntab * 128
    DZ = min((65535 - 124) // S, dzmax)
    B0 = 65535 - DZ * S - 124
    T = round_up(B0, 16)
    PL = 0 if plane_bytes <= B0 else round_up(T + (DZ + 1) * S, 16)
    total = T + (DZ + 1) * S if plane_bytes <= B0 else PL + plane_bytes
    return dict(S=S, DZ=DZ, B0=B0, T=T, PL=PL, total=total)


def joint_plane_bytes(R, waves=16):
    """Two RGBX planes of the joint kernel, 8 outputs per thread (Geom<R, 8, 16>)."""
    L = round_up(R, 4)
    s_words = round_up(128 + 2 * L, 8) + 4
    return 4 * 2 * (waves * 4 + 2 * R) * s_words


def check_addresses(lay, ntab, dmax, zero_from):
    """Every (d, k, c): the word read and the word meant agree; half-wave banks distinct."""
    S, DZ, B0, T = lay["S"], lay["DZ"], lay["B0"], lay["T"]
    d = np.arange(dmax + 1, dtype=np.int64)[:, None]
    c = np.arange(32, dtype=np.int64)[None, :]
    reg = np.minimum(d * S + B0 + 4 * c, 65535)
    for k in range(ntab):
        addr = reg + (T - B0) + 128 * k
        assert np.all(addr % 4 == 0)
        rel = addr - T
        dd, rem = rel // S, rel % S
        kk, cc = rem // 128, (rem % 128) // 4
        sat = d > DZ
        want_d = np.where(sat, DZ, d)
        assert np.all(kk == k)
        assert np.all(dd == np.broadcast_to(want_d, dd.shape))
        assert np.all(cc[~sat[:, 0]] == np.broadcast_to(c, cc.shape)[~sat[:, 0]])
        assert np.all(cc[sat[:, 0]] == 31)
        # unsaturated lanes of one half-wave: 32 distinct banks (ds_read_b32: bank = addr/4 mod 32)
        banks = (addr[: DZ + 1] // 4) % 32
        assert all(len(set(row)) == 32 for row in banks.tolist())
    assert zero_from <= DZ, "saturation must land on an exact-zero entry"


@pytest.mark.parametrize("R", range(1, 7))
def test_folded_jbf_addresses(R):
    ntab = len(disc_r2_values(R))
    lay = sat_layout(ntab, 31, joint_plane_bytes(R))
    assert lay["total"] <= LDS_BUDGET, "the 16-wave joint tile must fit with the tables"
    assert lay["T"] - lay["B0"] + (ntab - 1) * 128 <= 65535  # ds_read immediate
    assert lay["PL"] == 0 or lay["PL"] >= lay["T"] + (lay["DZ"] + 1) * lay["S"]  # tables below the planes
    for profile in (o.CUDA, o.CPP):
        wc = o.color_lut(768, SIGMA_TEXTURE, profile)
        zero_from = int(np.flatnonzero(wc)[-1]) + 1
        assert zero_from == 25 and not wc[zero_from:].any()
        check_addresses(lay, ntab, 765, zero_from)


def test_folded_jbf_radius_limit():
    """Beyond R = 6 the 16-bit range cannot hold 25 distances of the r^2 tables."""
    for R in range(1, 7):
        assert sat_layout(len(disc_r2_values(R)), 31, 0)["DZ"] >= 25
    assert sat_layout(len(disc_r2_values(7)), 31, 0)["DZ"] < 25


def test_adaptive_addresses():
    # one table, DZ = 511 -> B0 = 3, table at byte 16 (kAdaSatB0, kAdaSatT)
    lay = sat_layout(1, 511, 1 << 30)
    assert (lay["B0"], lay["T"]) == (3, 16)
    for profile in (o.CUDA, o.CPP):
        wc = o.color_lut(1536, 30.0, profile)
        zero_from = int(np.flatnonzero(wc)[-1]) + 1
        assert zero_from <= 511 and not wc[zero_from:].any()
        # dist = sum of three |(n - c) - o| <= 1530
        check_addresses(lay, 1, 1530, zero_from)
