"""CPU tests: the C-ABI library loads, exports every entry point include/vip.h
declares, and the Python mirror keeps the reference API surface. No compute call
is made here (there is no GPU in the CPU suite)."""
import inspect
import os
import re

import pytest

from conftest import ROOT


def _header_symbols():
    text = open(os.path.join(ROOT, "include", "vip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(vip_\w+)\s*\(", text, re.M)))


def test_library_exports_every_declared_symbol():
    import ctypes
    import various_image_processings_amd as vip
    handle = ctypes.CDLL(vip.LIB_PATH)
    syms = _header_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(handle, s)]
    assert not missing, missing


def test_python_binding_declares_every_symbol():
    from various_image_processings_amd import _lib
    assert sorted(_lib.SIGNATURES) == _header_symbols()


def test_abi_constants():
    import various_image_processings_amd as vip
    L = vip.lib()
    assert L.vip_abi_version() == 1
    assert L.vip_max_radius() == 15
    assert b"ksize" in L.vip_error_string(10002)
    assert L.vip_error_string(0) == b"success"


def test_bilateral_wave_knob_validates():
    """vip_bilateral_set_waves is host state only (no device call): 0 / 16 / 8 / 4 are
    accepted, anything else is VIP_ERR_INVALID_ARGUMENT."""
    import various_image_processings_amd as vip
    L = vip.lib()
    try:
        for w in (16, 8, 4, 0):
            assert L.vip_bilateral_set_waves(w) == 0
        for w in (12, 2, -1, 32):
            assert L.vip_bilateral_set_waves(w) == 10001
    finally:
        L.vip_bilateral_set_waves(0)


def test_reference_api_surface():
    """Same names and defaults as include/cuda/*.hpp of the reference."""
    import various_image_processings_amd as vip
    sig = inspect.signature(vip.CudaBilateralFilter.__init__)
    assert [sig.parameters[p].default for p in ("ksize", "sigma_space", "sigma_color")] == [9, 10.0, 30.0]
    sig = inspect.signature(vip.CudaAdaptiveBilateralFilter.__init__)
    assert [sig.parameters[p].default for p in ("ksize", "sigma_space", "sigma_color")] == [9, 10.0, 30.0]
    sig = inspect.signature(vip.CudaBilateralTextureFilter.__init__)
    assert [sig.parameters[p].default for p in ("ksize", "nitr")] == [9, 3]
    assert inspect.signature(vip.cuda_gradient).parameters["src_ch"].default == 1
    assert inspect.signature(vip.DeviceImage.__init__).parameters["channels"].default == 1
    for cls, methods in ((vip.CudaBilateralFilter, ("bilateral_filter", "joint_bilateral_filter")),
                         (vip.CudaAdaptiveBilateralFilter, ("execute",)),
                         (vip.CudaBilateralTextureFilter, ("execute",))):
        for m in methods:
            assert callable(getattr(cls, m))


def test_product_does_not_import_oracle():
    """The product package must not route through the CPU oracle."""
    pkg = os.path.join(ROOT, "various_image_processings_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".hpp", ".h")):
                text = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"(import\s+oracle|from\s+oracle|liboracle|vipo_)", text), f


def test_cpp_headers_mirror_reference_signatures():
    hdr = open(os.path.join(ROOT, "include", "cuda", "bilateral_filter.hpp")).read()
    assert "void bilateral_filter(const std::uint8_t* const d_src, std::uint8_t* const d_dst) const;" in hdr
    hdr = open(os.path.join(ROOT, "include", "cuda", "bilateral_texture_filter.hpp")).read()
    assert "void execute(const std::uint8_t* const d_src, std::uint8_t* const d_dst);" in hdr


@pytest.mark.parametrize("name", ["vip_benchmark", "vip_host_pipeline"])
def test_sample_links_against_library(name):
    """samples/* (C++ drop-in API consumers) are built and resolve libvip_hip.so."""
    import subprocess
    exe = os.path.join(ROOT, "samples", name)
    if not os.path.exists(exe):
        pytest.skip("sample not built (make -C various_image_processings_amd/csrc samples)")
    out = subprocess.run(["ldd", exe], capture_output=True, text=True).stdout
    line = [l for l in out.splitlines() if "libvip_hip" in l]
    assert line and "not found" not in line[0]
