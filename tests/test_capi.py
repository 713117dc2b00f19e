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
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(vip_\w+)\s*\(", text, re.M)))


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
    assert L.vip_max_radius() == 32
    assert b"ksize" in L.vip_error_string(10002)
    assert L.vip_error_string(0) == b"success"


def test_max_ksize_is_what_the_reference_runs():
    """The reference sizes dynamic shared memory from ksize with no cap, against CUDA's
    48 KB default (src/bilateral_filter_impl.cu:252-254, 272-275;
    src/adaptive_bilateral_filter_impl.cu:165-167): the largest ksize whose launch fits
    is what it runs. Recompute that bound from the reference's own smem formulas."""
    import various_image_processings_amd as vip
    L = vip.lib()
    smem = {  # bytes at ksize k: LUTs (k^2 + table) floats + (32 + k - 1)^2 * 3 per tile plane
        vip.VIP_FILTER_BILATERAL: lambda k: (k * k + 768) * 4 + (31 + k) ** 2 * 3,
        vip.VIP_FILTER_JOINT: lambda k: (k * k + 768) * 4 + 2 * (31 + k) ** 2 * 3,
        vip.VIP_FILTER_ADAPTIVE: lambda k: (k * k + 1536) * 4 + (31 + k) ** 2 * 3,
    }
    for f, fn in smem.items():
        kmax = max(k for k in range(1, 200, 2) if fn(k) <= 48 * 1024)
        assert L.vip_max_ksize(f) == kmax, (f, kmax)
    # texture: its JBF runs ksize 2k - 1 (src/bilateral_texture_filter_impl.cu:188)
    assert L.vip_max_ksize(vip.VIP_FILTER_TEXTURE) == (L.vip_max_ksize(vip.VIP_FILTER_JOINT) + 1) // 2 == 24
    assert L.vip_max_ksize(7) == 10001
    # ksize/2 of the largest accepted ksize
    assert L.vip_max_radius() == L.vip_max_ksize(vip.VIP_FILTER_BILATERAL) // 2


def test_stencil_path_knob_validates():
    import various_image_processings_amd as vip
    L = vip.lib()
    try:
        assert L.vip_set_stencil_path(vip.VIP_PATH_RUNTIME) == 0
        assert L.vip_set_stencil_path(vip.VIP_PATH_AUTO) == 0
        assert L.vip_set_stencil_path(2) == 10001
    finally:
        L.vip_set_stencil_path(vip.VIP_PATH_AUTO)


def test_texture_handle_holds_three_u8_frames():
    """A texture handle allocates two ping-pong frames and the guide (u8x3), no f32
    scratch: 75 MB at 4K instead of the reference Impl's 241 MB
    (src/bilateral_texture_filter_impl.cu:189-194)."""
    import various_image_processings_amd as vip
    L = vip.lib()
    assert L.vip_texture_scratch_bytes(3840, 2160) == 3 * 3840 * 2160 * 3
    assert L.vip_texture_scratch_bytes(0, 10) == 0


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
        for m in (0, 1, 2):
            assert L.vip_bilateral_set_wide(m) == 0
        for m in (3, -1):
            assert L.vip_bilateral_set_wide(m) == 10001
    finally:
        L.vip_bilateral_set_waves(0)
        L.vip_bilateral_set_wide(0)


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


def _shard_header_symbols():
    text = open(os.path.join(ROOT, "include", "vip_shard.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(vip_\w+)\s*\(", text, re.M)))


def test_shard_library_exports_and_binds_every_symbol():
    """libvip_shard.so (include/vip_shard.h) loads here (RCCL without a GPU) and exports
    every declared entry point; the Python binding declares the same set."""
    import ctypes
    from various_image_processings_amd import _shard_lib
    syms = _shard_header_symbols()
    assert len(syms) >= 9
    handle = ctypes.CDLL(_shard_lib.LIB_PATH)
    assert not [s for s in syms if not hasattr(handle, s)]
    assert sorted(_shard_lib.SIGNATURES) == syms
    _shard_lib.lib()


def test_native_rows_match_slab_geometry():
    from various_image_processings_amd.sharded import native_rows, shard_rows
    for h in (1, 7, 2160, 16384, 16385):
        for n in (1, 2, 3, 5, 8):
            if h < n:
                continue
            rows = [native_rows(h, n, r) for r in range(n)]
            assert rows == [shard_rows(h, n, r) for r in range(n)]
            assert rows[0][0] == 0 and rows[-1][1] == h
            assert all(a[1] == b[0] for a, b in zip(rows, rows[1:]))


def test_shard_create_validates_before_device_work():
    """Bad kind / thin shards / bad ranks are rejected before any device or RCCL call
    (no GPU here), identically on every rank."""
    import ctypes
    from various_image_processings_amd import _shard_lib as S
    L = S.lib()
    h = ctypes.c_void_p()
    idb = ctypes.create_string_buffer(128)
    args = lambda kind, fh, k, n, r: (ctypes.byref(h), kind, 64, fh, k, 10.0, 30.0, 0, n, r, idb, 1000)  # noqa: E731
    assert L.vip_shard_create(*args(3, 100, 15, 2, 0)) == 10001      # texture is not a shard kind
    assert L.vip_shard_create(*args(0, 100, 31, 8, 0)) == 10001      # 12-row shards < 15-row halo
    assert L.vip_shard_create(*args(0, 100, 15, 2, 2)) == 10001      # rank outside the world
    assert L.vip_shard_create(*args(0, 100, 8, 2, 0)) == 10002       # even ksize
    assert L.vip_shard_create(ctypes.byref(h), 0, 64, 100, 15, 10.0, 30.0, 0, 2, 0, None, 1000) == 10001


def test_launch_log_names_kernels_like_the_profiler():
    """vip_launched_kernels (no GPU needed): a kernel handle noted by the launch path comes
    back as the profiler names it (demangled, template arguments, no parameter list), each
    once; a size query keeps the list, a read clears it."""
    import ctypes
    from various_image_processings_amd import _lib
    from various_image_processings_amd.filters import launched_kernels
    lib = _lib.lib()
    libdl = ctypes.CDLL(None)
    libdl.dlsym.restype = ctypes.c_void_p
    libdl.dlsym.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    handle = libdl.dlsym(lib._handle, b"_ZN3vip16bilateral_kernelILi7ELi16ELb0ELb1ELi32ELi8ELi768ELb0ELi16ELb0EEEvNS_11StencilArgsE")
    assert handle
    note = lib._ZN3vip11note_launchEPKv
    note.argtypes = [ctypes.c_void_p]
    launched_kernels()
    note(handle)
    note(handle)
    assert lib.vip_launched_kernels(None, 0) > 0
    assert launched_kernels() == ["void vip::bilateral_kernel<7, 16, false, true, 32, 8, 768, false, 16, false>"]
    assert launched_kernels() == []


def test_build_stamp_matches_the_tree():
    """__graft_entry__.build() stamps the libraries with the sources they were built from
    (various_image_processings_amd/build_info.json); bench.py reports the check as `build`.
    In a built tree whose sources are unchanged, the libraries on disk are the stamped ones."""
    from various_image_processings_amd import build_info
    c = build_info.check()
    if c.get("stamp", 1) is None:
        pytest.skip("not built by __graft_entry__.build() in this tree")
    assert set(c) >= {"sources_match", "libs_match", "built_utc"}
    if c["sources_match"]:
        assert c["libs_match"], c
    assert len(build_info.source_files()) > 15


def test_build_stamp_missing_library_is_a_mismatch(tmp_path, monkeypatch):
    """A library missing both when the stamp was written and now is not a match,
    and a stamp without a `libs` entry is a mismatch, not a KeyError."""
    import json
    from various_image_processings_amd import build_info
    info = tmp_path / "build_info.json"
    monkeypatch.setattr(build_info, "INFO", str(info))
    monkeypatch.setattr(build_info, "_lib_sha", lambda name: None)
    info.write_text(json.dumps(dict(sources_sha256="x", libs={n: None for n in build_info.LIBS})))
    assert build_info.check()["libs_match"] is False
    info.write_text(json.dumps(dict(sources_sha256="x")))
    assert build_info.check()["libs_match"] is False


def test_kernel_timing_validates_before_device_work():
    """vip_kernel_timing_*: capacity outside 1..65536 is refused before any device call; a read
    with nothing recorded (or while recording) is refused; end reports the launches recorded."""
    import ctypes
    from various_image_processings_amd import _lib
    lib = _lib.lib()
    assert lib.vip_kernel_timing_begin(0) == 10001
    assert lib.vip_kernel_timing_begin(1 << 17) == 10001
    assert lib.vip_kernel_timing_end() == 0
    ms = ctypes.c_float()
    assert lib.vip_kernel_timing_get(0, ctypes.byref(ms), None, 0) == 10001
    assert lib.vip_kernel_timing_get(-1, ctypes.byref(ms), None, 0) == 10001
